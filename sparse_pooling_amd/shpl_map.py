"""Device-side correspondence matrix M and the SHPL pulls (torch plumbing over
the libshpl C ABI).

``ShplMap`` is M resident in HBM as four flat arrays over global ids (so one
map can hold a whole batch of frames):

* ``cell[e]``  BEV row of entry e (M row, frame offset included)
* ``col[e]``   column k of entry e (None = identity, as the index builder emits)
* ``val[e]``   M value (f32, what TF's float32 placeholder holds)
* ``pix[k]``   image pixel of column k (img_index_flip row, frame offset included)

plus the destination-keyed CSRs built from it on demand. The pulls that use
them implement the reference ops (avod/avod/utils/sparse_pool_utils.py:61-117)
and their TF gradients.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L
from .errors import InvalidArgumentError


def _i32(n, device):
    return torch.empty(max(int(n), 1), dtype=torch.int32, device=device)


_SIDE = {}  # device -> the side stream of ShplMap.prefetch_csr


def raise_for_bits(bits):
    """The exception a device error word's bits (SHPL_EBIT_*) stand for, raised; nothing for 0."""
    if not bits:
        return
    what = []
    if bits & L.EBIT_ROW:
        what.append("M row index outside [0, M_size[0])")
    if bits & L.EBIT_COL:
        what.append("M column index outside [0, M_size[1])")
    if bits & L.EBIT_PIXEL:
        what.append("source index (b, v, u) outside the feature map")
    if bits & L.EBIT_VALUES:
        what.append("number of M values does not match number of indices")
    if bits & L.EBIT_CAPACITY:
        what.append("a frame holds more points than max_points_per_frame")
    if bits & L.EBIT_BARRIER:  # not an input error: the one-launch index build could not proceed
        raise RuntimeError("shpl_build_index_buckets: a frame barrier gave up (chunks not resident) or "
                           "found its words not zeroed; the step's results are invalid")
    raise InvalidArgumentError("; ".join(what))


class ShplMap:
    """M on the device. Entries are grouped by frame: frame f owns entry slots
    [frame_off[f], frame_off[f+1]) of which the first frame_nnz[f] are live
    (frame_nnz None: all), BEV rows [f*n_cells/F, (f+1)*n_cells/F) and image
    pixels [f*n_pix/F, (f+1)*n_pix/F)."""

    def __init__(self, cell, col, val, pix, nnz_cap, n_cells, n_pix, n_cols, device,
                 frame_off=None, frame_nnz=None, n_frames=1, err=None):
        self.cell, self.col, self.val, self.pix = cell, col, val, pix
        self.nnz_cap = int(nnz_cap)
        self.n_cells = int(n_cells)
        self.n_pix = int(n_pix)
        self.n_cols = int(n_cols)
        self.device = device
        self.n_frames = int(n_frames)
        if frame_off is None:
            frame_off = torch.tensor([0, self.nnz_cap], dtype=torch.int64, device=device)
        self.frame_off, self.frame_nnz = frame_off, frame_nnz
        self.err = err if err is not None else torch.zeros(1, dtype=torch.int32, device=device)
        self._csr = {}
        self._pending = {}  # key -> event of a csr() built on a side stream (prefetch_csr)

    # ---------------------------------------------------------------- checks
    def error_bits(self):
        return int(self.err.item()) & 0xFFFFFFFF

    def check(self):
        """Raise like TF-CPU's InvalidArgumentError if any index was invalid
        (one device->host read of the error word)."""
        raise_for_bits(self.error_bits())

    # ------------------------------------------------------------------ CSR
    # Row-keyed pulls (shpl_csr.key_range: one launch per pull) for maps of fewer
    # than ROWS_FRAMES frames with at most ROWS_MAX_KEYS destinations per frame;
    # ROW_PULLS = True / False forces the form (tests).
    ROWS_FRAMES, ROWS_MAX_KEYS, ROWS_MAX_CAP = 32, 65536, 1 << 24
    ROW_PULLS = None
    # shpl_build_csr_path's builder for the flat CSRs (L.CSR_AUTO: the library's choice by batch shape)
    CSR_PATH = L.CSR_AUTO

    def csr(self, direction, order):
        key = (direction, order)
        if key in self._csr:
            c = self._csr[key]
            if key in self._pending:  # built on a side stream: the current one waits for it, and owns its buffers
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(self._pending.pop(key))
                for t in (c.ent_dst, c.ent_src, c.ent_val, c.ent_col, c.key_range, c.ws):
                    if t is not None:
                        t.record_stream(cur)
            return c
        n_keys = self.n_cells if direction == L.BY_CELL else self.n_pix
        rows = self.ROW_PULLS
        if rows is None:
            # (the range CSR carries entry offsets in 24 bits: capacities under 2^24 slots)
            rows = (self.n_frames < self.ROWS_FRAMES and n_keys // max(self.n_frames, 1) <= self.ROWS_MAX_KEYS
                    and self.nnz_cap < self.ROWS_MAX_CAP)
        c = L.Csr(n_keys, self.nnz_cap, self.device, with_col=direction == L.BY_PIXEL, key_range=rows)
        L.check(L.lib().shpl_build_csr_path(self.CSR_PATH, direction, order, self.n_frames, L.ptr(self.frame_off),
                                            L.ptr(self.frame_nnz), n_keys // self.n_frames,
                                            L.ptr(self.cell), L.ptr(self.col), L.ptr(self.val),
                                            L.ptr(self.pix), c.ref(), L.ptr(c.ws), c.ws.numel(),
                                            L.stream_of(self.device)), "shpl_build_csr_path")
        self._csr[key] = c
        return c

    def prefetch_csr(self, direction, order):
        """Start csr(direction, order) on a side stream (after the current stream's work so far: the
        map's arrays); the first csr() of that key later makes its stream wait for it. The training
        forward of FusionConv.fused starts the pixel-keyed CSR of the image gradient this way, so that it
        sorts beside the forward conv instead of on the backward's critical path."""
        key = (direction, order)
        if key in self._csr or torch.cuda.is_current_stream_capturing():
            return
        dev = torch.device(self.device)
        side = _SIDE.get(dev)
        if side is None:
            side = _SIDE[dev] = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        for t in (self.cell, self.col, self.val, self.pix, self.frame_off, self.frame_nnz):
            if isinstance(t, torch.Tensor):
                t.record_stream(side)  # read there: not reused before the side stream is done with them
        with torch.cuda.stream(side):
            self.csr(direction, order)
            ev = torch.cuda.Event()
            ev.record(side)
        self._pending[key] = ev

    def csr_tensors(self, direction, order):
        """(ent_dst, ent_src, ent_val, ent_col or None) of csr(direction, order):
        the CSR as the tensors the torch.ops.shpl operators take (ops.py)."""
        c = self.csr(direction, order)
        return c.ent_dst, c.ent_src, c.ent_val, c.ent_col


def pack_map(mij, values, m_size, idx, img_shape, validate=True):
    """Reference-format M (Mij [nnz,2] i64, M_val [nnz], M_size [2]) and the
    gather index img_index_flip [ncols,3] -> ShplMap (single frame, as the
    reference's batch-1 graphs)."""
    dev = idx.device
    mij = mij.to(device=dev, dtype=torch.int64).reshape(-1, 2).contiguous()
    values = values.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    if idx.dtype not in (torch.int32, torch.int64):
        idx = idx.to(torch.int64)
    idx = idx.reshape(-1, 3).contiguous()
    R, ncols = int(m_size[0]), int(m_size[1])
    if ncols != idx.shape[0]:
        raise InvalidArgumentError(
            f"Cannot multiply A and B because inner dimension does not match: {ncols} vs. {idx.shape[0]}")
    nnz = mij.shape[0]
    B, H, W = (int(s) for s in img_shape[:3])
    cell, col = _i32(nnz, dev), _i32(nnz, dev)
    val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    pix = _i32(ncols, dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L.check(L.lib().shpl_pack_map(nnz, L.ptr(mij), L.ptr(values), values.numel(), R, ncols,
                                  L.ptr(idx), L.I64 if idx.dtype == torch.int64 else L.I32,
                                  B, H, W, 0, 0, 0, L.ptr(cell), L.ptr(col), L.ptr(val), L.ptr(pix),
                                  L.ptr(err), L.stream_of(dev)), "shpl_pack_map")
    m = ShplMap(cell, col, val, pix, nnz, R, B * H * W, ncols, dev, err=err)
    if validate:
        m.check()
    return m


# -------------------------------------------------------------------- pulls

def pull(smap, direction, order, src, src_stride, src_off, c_pool, out, out_stride,
         pass_=None, pass_stride=0, pass_off=0, c_pass=0, mode=L.OUT_POOL, part=None):
    """shpl_pull through smap's CSR; part "dense" / "sparse": only shpl_pull_dense (the pass-through chunks and
    the pooled chunks' zeros, no index read) or shpl_pull_sparse (the pooled rows over them), which together
    give shpl_pull's output bit for bit -- so the dense half can run early, on another stream. part "once":
    shpl_pull_once (OUT_POOL over a CSR with key ranges: every row written once, the zeros included)."""
    c = smap.csr(direction, order)
    fn, name = {None: (L.lib().shpl_pull, "shpl_pull"), "dense": (L.lib().shpl_pull_dense, "shpl_pull_dense"),
                "sparse": (L.lib().shpl_pull_sparse, "shpl_pull_sparse"),
                "once": (L.lib().shpl_pull_once, "shpl_pull_once")}[part]
    L.check(fn(direction, L.dtype_code(out), c.ref(), L.ptr(src), src_stride, src_off, c_pool, L.ptr(pass_),
               pass_stride, pass_off, c_pass, mode, L.ptr(out), out_stride, L.stream_of(out.device)), name)
    return out


def op_pull(smap, direction, order, src, out_shape, src_off=0, c_pool=None, pass_=None, pass_off=0, c_pass=None,
            mode=L.OUT_POOL):
    """torch.ops.shpl.pull through smap's CSR (ops.py): a new output tensor."""
    from . import ops  # noqa: F401 -- registers torch.ops.shpl
    c_pool = int(src.shape[-1]) - src_off if c_pool is None else int(c_pool)
    if c_pass is None:
        c_pass = 0 if pass_ is None else int(pass_.shape[-1]) - pass_off
    return torch.ops.shpl.pull(src, *smap.csr_tensors(direction, order), direction, [int(v) for v in out_shape],
                               int(src_off), c_pool, pass_, int(pass_off), int(c_pass), mode)


def pool_img_to_bev(smap, img, bev_shape, bev=None):
    """img [.., Ci] -> [B,Hb,Wb,Ci] (or [bev || pooled] when ``bev`` is given)."""
    Ci = img.shape[-1]
    if bev is None:
        return op_pull(smap, L.BY_CELL, L.ORDER_ENTRY, img, tuple(bev_shape[:3]) + (Ci,))
    Cb = bev.shape[-1]
    return op_pull(smap, L.BY_CELL, L.ORDER_ENTRY, img, tuple(bev.shape[:3]) + (Cb + Ci,), pass_=bev,
                   mode=L.OUT_CONCAT)


def pool_bev_to_img(smap, bev, img_shape, img=None):
    """bev [.., Cb] -> [B,Hi,Wi,Cb] (or [img || pooled] when ``img`` is given)."""
    Cb = bev.shape[-1]
    if img is None:
        return op_pull(smap, L.BY_PIXEL, L.ORDER_COL_ROW, bev, tuple(img_shape[:3]) + (Cb,))
    Ci = img.shape[-1]
    return op_pull(smap, L.BY_PIXEL, L.ORDER_COL_ROW, bev, tuple(img.shape[:3]) + (Ci + Cb,), pass_=img,
                   mode=L.OUT_CONCAT)


# ------------------------------------------------------------------ autograd

def _c(t):
    return t if t.is_contiguous() else t.contiguous()


class _PoolConcatFn(torch.autograd.Function):
    """bv_fused = tf.concat([bev, _sparse_pool_op(M, img, idx, .)], axis=3)
    (sparse_pool_utils.py:65-72), the concat fused into the pull."""

    @staticmethod
    def forward(ctx, bev, img, smap):
        bev, img = _c(bev), _c(img)
        ctx.smap, ctx.Cb, ctx.img_shape = smap, bev.shape[-1], img.shape
        return pool_img_to_bev(smap, img, bev.shape, bev=bev)

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        Cb, Ci = ctx.Cb, ctx.img_shape[-1]
        d_img = op_pull(ctx.smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, g, ctx.img_shape, src_off=Cb, c_pool=Ci)
        return g[..., :Cb].contiguous(), d_img, None


class _DualFn(torch.autograd.Function):
    """Dual SHPL (sparse_pool_layer with bv_index set, sparse_pool_utils.py:61-92):

    forward : bv_fused  = [bev || pool(img)],  img_fused = [img || trans(bev)]
    backward: TF's gradient with the concat split and the add_n of the two
              paths into each input fused into one pull per input (OUT_ADD).
    """

    @staticmethod
    def forward(ctx, bev, img, smap):
        bev, img = _c(bev), _c(img)
        ctx.smap, ctx.Cb, ctx.Ci = smap, bev.shape[-1], img.shape[-1]
        ctx.bev_shape, ctx.img_shape = bev.shape, img.shape
        return (pool_img_to_bev(smap, img, bev.shape, bev=bev),
                pool_bev_to_img(smap, bev, img.shape, img=img))

    @staticmethod
    def backward(ctx, g_bv, g_img):
        smap, Cb, Ci = ctx.smap, ctx.Cb, ctx.Ci
        if g_bv is not None:
            g_bv = _c(g_bv)
        if g_img is not None:
            g_img = _c(g_img)
        # d_bev = g_bv[..., :Cb] + matmul(sparse_transpose(M), gather_nd(g_img[..., Ci:]), adjoint_a)
        if g_img is None:
            d_bev = g_bv[..., :Cb].contiguous()
        else:
            d_bev = op_pull(smap, L.BY_CELL, L.ORDER_COL_ENTRY, g_img, ctx.bev_shape, src_off=Ci, c_pool=Cb,
                            pass_=g_bv, c_pass=Cb, mode=L.OUT_POOL if g_bv is None else L.OUT_ADD)
        # d_img = g_img[..., :Ci] + scatter_nd(idx, matmul(M, g_bv[..., Cb:], adjoint_a))
        if g_bv is None:
            d_img = g_img[..., :Ci].contiguous()
        else:
            d_img = op_pull(smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, g_bv, ctx.img_shape, src_off=Cb, c_pool=Ci,
                            pass_=g_img, c_pass=Ci, mode=L.OUT_POOL if g_img is None else L.OUT_ADD)
        return d_bev, d_img, None


def layer(bev, img, smap, dual=False):
    """(bv_fused, img_fused) of sparse_pool_layer for a packed map."""
    if dual:
        return _DualFn.apply(bev, img, smap)
    return _PoolConcatFn.apply(bev, img, smap), img


def pool_op(img, smap, bev_shape):
    """_sparse_pool_op: torch.ops.shpl.spmm (ops.py), gradient = the pixel-keyed pull."""
    from . import ops
    return ops.sparse_pool(_c(img), smap, tuple(bev_shape))


def trans_op(bev, smap, img_shape):
    """_sparse_pool_trans_op: torch.ops.shpl.spmm, gradient = the cell-keyed pull."""
    from . import ops
    return ops.sparse_pool_trans(_c(bev), smap, tuple(img_shape))


# --------------------------------------------------------------- index build

class IndexBatch:
    """Result of the fused device index builder over a batch of frames."""

    def __init__(self, smap, mij, flip, frame_nnz, frame_off, n_frames, bev_hw, img_hw):
        self.map = smap
        self.mij, self.flip = mij, flip
        self.frame_nnz, self.frame_off = frame_nnz, frame_off
        self.n_frames = n_frames
        self.bev_hw, self.img_hw = bev_hw, img_hw


def build_index_batch(points, voxels, point_offsets, P, im_size, bv_size, stride, max_points,
                      mval=None, ref_outputs=False, ws=None, point_counts=None):
    """Fused gen_sparse_pooling_input_avod + produce_sparse_pooling_input for a
    batch of frames in one pass (shpl_build_index). All inputs are device
    tensors; nothing synchronises the host."""
    dev = points.device
    points, point_offsets, P = points.contiguous(), point_offsets.contiguous(), P.contiguous()
    if voxels.stride(1) != 1:
        voxels = voxels.contiguous()
    n_frames = int(point_offsets.numel()) - 1
    N = int(points.shape[0])
    s_img, s_bv = float(stride[0]), float(stride[1])
    wq, hq = int(np.floor(im_size[0] / s_img)), int(np.floor(im_size[1] / s_img))
    bhq, bwq = int(np.floor(bv_size[0] / s_bv)), int(np.floor(bv_size[1] / s_bv))
    cell, pix = _i32(N, dev), _i32(N, dev)
    val = torch.empty(max(N, 1), dtype=torch.float32, device=dev)
    mij = torch.empty((max(N, 1), 2), dtype=torch.int64, device=dev) if ref_outputs else None
    flip = torch.empty((max(N, 1), 3), dtype=torch.int64, device=dev) if ref_outputs else None
    frame_nnz = torch.empty(n_frames, dtype=torch.int64, device=dev)
    frame_off = torch.empty(n_frames + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    if ws is None:
        ws = L.workspace(L.index_ws_bytes(n_frames, max_points), dev)
    pdt = L.F64 if points.dtype == torch.float64 else L.F32
    vit = L.I64 if voxels.dtype == torch.int64 else L.I32
    L.check(L.lib().shpl_build_index(n_frames, L.ptr(point_offsets), L.ptr(point_counts), int(max_points),
                                     L.ptr(points),
                                     pdt, L.ptr(voxels), vit, int(voxels.stride(0)), L.ptr(P),
                                     float(im_size[0]), float(im_size[1]), float(bv_size[0]),
                                     float(bv_size[1]), s_img, s_bv, L.ptr(mval), L.ptr(cell),
                                     L.ptr(pix), L.ptr(val), L.ptr(mij), L.ptr(flip),
                                     L.ptr(frame_nnz), L.ptr(frame_off), L.ptr(err), L.ptr(ws),
                                     ws.numel(), L.stream_of(dev)), "shpl_build_index")
    smap = ShplMap(cell, None, val, pix, N, n_frames * bhq * bwq, n_frames * hq * wq, N, dev,
                   frame_off=frame_off, frame_nnz=frame_nnz, n_frames=n_frames, err=err)
    return IndexBatch(smap, mij, flip, frame_nnz, frame_off, n_frames, (bhq, bwq), (hq, wq))
