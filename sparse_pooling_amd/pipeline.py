"""Preallocated batched SHPL pipeline: the per-step hot path of the bench.

One step over a batch of B frames (all inputs already in HBM):

1. ``shpl_build_index`` -- points + voxel indices + P of every frame ->
   M (cell, pix, val) and per-frame entry counts (a1-a4, one pass);
2. ``shpl_build_csr``   -- BEV-cell-keyed CSR of M, TF nnz order;
3. ``shpl_pull``        -- bv_fused = [bev || pool(img)] for all frames
   (a8 + the concat of a10), the dominant, HBM-bound kernel.

Buffers are sized once for the largest frame; nothing allocates or
synchronises inside ``step``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L
from .shpl_map import ShplMap, raise_for_bits


class FusedPipeline:
    # row-keyed pulls (one launch per pull, shpl_csr.key_range) for batches under this many frames whose
    # maps have at most ROWS_MAX_KEYS destinations per frame: latency-bound layers (config 3)
    ROWS_FRAMES, ROWS_MAX_KEYS, ROWS_MAX_CAP = 32, 65536, 1 << 24
    # bucketed pixel-keyed CSRs with ent_col (per-column partials in the pulls; A/B of the identity-column form)
    PIXEL_COLS = False
    # split: the pooled half by shpl_pull_once (k_sparse's walk + the empty rows' zeros, one launch); False: the
    # row-keyed k_rows (1.11 ms per 64 frames at config 6, a wave per 1 KB row: latency-bound)
    SPLIT_ONCE = True
    # bucketed CSRs: run heads of this many entries per destination (shpl_csr.heads; 0 = none): the row-keyed
    # pulls read a row's first entries in the round trip of its key_range
    HEAD_K = 8

    def __init__(self, n_frames, max_points_per_frame, total_points, im_size, bv_size, stride,
                 c_bev, c_img, dtype=torch.float32, device="cuda", dual=False, rows=None, live=False,
                 buckets=None, split=False):
        """live: the sparse passes walk each frame's live entries (shpl_csr frame layout) instead of the
        whole capacity -- for capacities far above the entry counts (FramePipeline: raw-scan slots per
        voxel point); at config 2 (capacity = entries) the capacity walk is faster (2.22 vs 2.24 ms).
        buckets (default: with rows): the index build also cuts M into destination buckets
        (shpl_build_index_buckets), one launch sorts both CSRs out of them (shpl_build_csr_buckets) and
        each pull pair is one row-keyed launch (shpl_pull_pair), all on one stream; the forward's
        pass-through halves ride the index launches.
        rows without buckets: the range CSRs (one launch per key) + one k_rows launch per pull,
        on two streams.
        split (img->BEV only): the two halves of bv_fused by two passes that need not wait for each other --
        the pass-through copy (no index) beside the index chain, and the pooled half written once, zeros
        included, by a row-keyed pull over the frame CSR's key ranges right after the chain (no k_dense zeros
        for k_sparse to overwrite). For wide channels (config 6: 1 KB halves), where writing half rows costs
        nothing over whole ones."""
        dev = torch.device(device)
        self.split = bool(split)
        if self.split:
            assert not dual, "split: the img->BEV layer"
            rows, buckets = False, False
        self.dev, self.dtype, self.dual = dev, dtype, dual
        self.B = int(n_frames)
        self.max_points = int(max_points_per_frame)
        self.N = int(total_points)
        self.im_size, self.bv_size = tuple(im_size), tuple(bv_size)
        self.stride = (float(stride[0]), float(stride[1]))
        self.Cb, self.Ci = int(c_bev), int(c_img)
        self.Hb = int(np.floor(bv_size[0] / self.stride[1]))
        self.Wb = int(np.floor(bv_size[1] / self.stride[1]))
        self.Hi = int(np.floor(im_size[1] / self.stride[0]))
        self.Wi = int(np.floor(im_size[0] / self.stride[0]))
        self.n_cells = self.B * self.Hb * self.Wb
        self.n_pix = self.B * self.Hi * self.Wi
        if rows is None:
            rows = (self.B < self.ROWS_FRAMES and max(self.Hb * self.Wb, self.Hi * self.Wi) <= self.ROWS_MAX_KEYS
                    and self.N < self.ROWS_MAX_CAP)  # the range CSR's 24-bit entry offsets
        self.rows = bool(rows)
        self.buckets = self.rows if buckets is None else bool(buckets) and self.rows
        # dual layers in step_overlapped: the cell-keyed sparse pass beside img_fused's stream
        self.interleave = True
        N = max(self.N, 1)
        i32 = dict(dtype=torch.int32, device=dev)
        self.cell = torch.empty(N, **i32)
        self.pix = torch.empty(N, **i32)
        self.val = torch.empty(N, dtype=torch.float32, device=dev)
        self.frame_nnz = torch.empty(self.B, dtype=torch.int64, device=dev)
        self.frame_off = torch.empty(self.B + 1, dtype=torch.int64, device=dev)
        self.err = torch.zeros(1, **i32)
        self.index_ws = L.workspace(L.index_ws_bytes(self.B, self.max_points), dev)
        # rows pulls: with key_range
        head_k = self.HEAD_K if self.buckets else 0
        self.csr = L.Csr(self.n_cells, self.N, dev, with_col=False,
                         key_range=self.rows or self.split, head_k=head_k)  # BEV-cell CSR (img -> BEV)
        self.bv_fused = torch.empty((self.B, self.Hb, self.Wb, self.Cb + self.Ci), dtype=dtype, device=dev)
        if dual:
            # pixel CSR (BEV -> img); from the buckets without ent_col: every entry its own column (shpl.h)
            with_col = not self.buckets or self.PIXEL_COLS
            self.pcsr = L.Csr(self.n_pix, self.N, dev, with_col=with_col, key_range=self.rows,
                              identity_cols=not with_col, head_k=head_k)
            self.img_fused = torch.empty((self.B, self.Hi, self.Wi, self.Ci + self.Cb), dtype=dtype,
                                         device=dev)
        if live:
            for c in (self.csr, self.pcsr if dual else None):
                if c is not None:
                    c.live_frames(self.frame_off, self.frame_nnz)
        self._lib = L.lib()
        if self.buckets:
            # zeroed once: its frame barrier words start at zero (every call leaves them so)
            self.bkt_ws = L.bucket_workspace(self.B, self.max_points, self.N, self.Hb * self.Wb, self.Hi * self.Wi,
                                             dev)
            self.bkt = L.ShplBuckets(self.B, self.max_points, self.N, self.Hb * self.Wb, self.Hi * self.Wi,
                                     self.frame_off.data_ptr(), self.frame_nnz.data_ptr(), self.cell.data_ptr(),
                                     self.pix.data_ptr(), self.val.data_ptr(), self.bkt_ws.data_ptr(),
                                     self.bkt_ws.numel(), self.err.data_ptr())

    # ------------------------------------------------------------------ steps
    def build_index(self, points, voxels, point_offsets, P, mval=None, point_counts=None, pass_copies=None):
        """pass_copies (bucketed pipelines): (bev, img) -- the forward's pass-through halves ride the index
        launches (shpl_pass_copy)."""
        assert points.is_contiguous() and point_offsets.is_contiguous() and P.is_contiguous()
        assert voxels.stride(1) == 1, "voxel rows must be contiguous"
        st = L.stream_of(self.dev)
        if self.buckets:
            L.check(self._lib.shpl_build_index_buckets(
                self.B, L.ptr(point_offsets), L.ptr(point_counts), self.max_points, L.ptr(points),
                L.F64 if points.dtype == torch.float64 else L.F32, L.ptr(voxels),
                L.I64 if voxels.dtype == torch.int64 else L.I32, int(voxels.stride(0)), L.ptr(P),
                float(self.im_size[0]), float(self.im_size[1]), float(self.bv_size[0]),
                float(self.bv_size[1]), self.stride[0], self.stride[1], L.ptr(mval), L.ptr(self.cell),
                L.ptr(self.pix), L.ptr(self.val), L.ptr(self.frame_nnz), L.ptr(self.frame_off),
                L.ptr(self.err), L.ptr(self.index_ws), self.index_ws.numel(), self.N, L.ptr(self.bkt_ws),
                self.bkt_ws.numel(), *self._copy_riders(pass_copies), st), "shpl_build_index_buckets")
            return
        L.check(self._lib.shpl_build_index(
            self.B, L.ptr(point_offsets), L.ptr(point_counts), self.max_points, L.ptr(points),
            L.F64 if points.dtype == torch.float64 else L.F32, L.ptr(voxels),
            L.I64 if voxels.dtype == torch.int64 else L.I32, int(voxels.stride(0)), L.ptr(P),
            float(self.im_size[0]), float(self.im_size[1]), float(self.bv_size[0]),
            float(self.bv_size[1]), self.stride[0], self.stride[1], L.ptr(mval), L.ptr(self.cell),
            L.ptr(self.pix), L.ptr(self.val), None, None, L.ptr(self.frame_nnz), L.ptr(self.frame_off),
            L.ptr(self.err), L.ptr(self.index_ws), self.index_ws.numel(), st), "shpl_build_index")

    # shpl_build_csr_path's builder (L.CSR_AUTO: chosen by batch shape; tests force the others)
    csr_path = L.CSR_AUTO

    def build_csr(self, which=("cell", "pixel")):
        st = L.stream_of(self.dev)
        if self.buckets:  # both CSRs from the index build's buckets, one launch
            L.check(self._lib.shpl_build_csr_buckets(
                ctypes.byref(self.bkt), self.csr.ref() if "cell" in which else None,
                self.pcsr.ref() if self.dual and "pixel" in which else None, st), "shpl_build_csr_buckets")
            return
        args = (self.B, L.ptr(self.frame_off), L.ptr(self.frame_nnz))
        if "cell" in which:
            L.check(self._lib.shpl_build_csr_path(
                L.CSR_FRAME if self.split else self.csr_path, L.BY_CELL, L.ORDER_ENTRY, *args, self.Hb * self.Wb, L.ptr(self.cell), None, L.ptr(self.val),
                L.ptr(self.pix), self.csr.ref(), L.ptr(self.csr.ws), self.csr.ws.numel(), st), "shpl_build_csr")
        if self.dual and "pixel" in which:
            L.check(self._lib.shpl_build_csr_path(
                self.csr_path, L.BY_PIXEL, L.ORDER_COL_ROW, *args, self.Hi * self.Wi, L.ptr(self.cell), None, L.ptr(self.val),
                L.ptr(self.pix), self.pcsr.ref(), L.ptr(self.pcsr.ws), self.pcsr.ws.numel(), st),
                "shpl_build_csr")

    def _pull(self, fn, csr, direction, src, cs, pass_, cp, out, st):
        L.check(fn(direction, L.dtype_code(out), csr.ref(), L.ptr(src), cs, 0, cs, L.ptr(pass_), cp, 0, cp,
                   L.OUT_CONCAT, L.ptr(out), cs + cp, st), "shpl_pull")

    def layer_dense(self, bev, img, which=("cell", "pixel")):
        """Streaming half of the layer (needs no M): pass-through copy + zeros.
        Row-keyed pulls (self.rows) have no separate streaming half; split: the pass-through copy alone."""
        if self.split:
            self._pass_copies(bev, img, ("cell",))
            return
        if self.rows:
            return
        st = L.stream_of(self.dev)
        if "cell" in which:
            self._pull(self._lib.shpl_pull_dense, self.csr, L.BY_CELL, img, self.Ci, bev, self.Cb, self.bv_fused,
                       st)
        if self.dual and "pixel" in which:
            self._pull(self._lib.shpl_pull_dense, self.pcsr, L.BY_PIXEL, bev, self.Cb, img, self.Ci,
                       self.img_fused, st)

    def _sparse(self, args):
        """shpl_pull_sparse(*args) on the current stream; with row-keyed CSRs the
        whole pull (shpl_pull's one launch)."""
        if self.rows:
            L.check(self._lib.shpl_pull(*args, L.stream_of(self.dev)), "shpl_pull")
            return
        L.check(self._lib.shpl_pull_sparse(*args, L.stream_of(self.dev)), "shpl_pull_sparse")

    def _concat_args(self, csr, direction, src, cs, pass_, cp, out):
        return (direction, L.dtype_code(out), csr.ref(), L.ptr(src), cs, 0, cs, L.ptr(pass_), cp, 0, cp,
                L.OUT_CONCAT, L.ptr(out), cs + cp)

    def _pull_pair(self, cell_desc, pix_desc):
        L.check(self._lib.shpl_pull_pair(self.csr.ref(), ctypes.byref(cell_desc) if cell_desc else None,
                                         self.pcsr.ref() if self.dual else None,
                                         ctypes.byref(pix_desc) if pix_desc else None,
                                         L.stream_of(self.dev)), "shpl_pull_pair")

    def _copy_riders(self, pass_copies):
        if pass_copies is None:
            return None, None
        bev, img = pass_copies
        dt = L.dtype_code(self.bv_fused)
        cell = L.ShplPassCopy(dt, bev.data_ptr(), self.Cb, self.bv_fused.data_ptr(), self.Cb + self.Ci, self.Cb)
        pix = L.ShplPassCopy(dt, img.data_ptr(), self.Ci, self.img_fused.data_ptr(), self.Ci + self.Cb,
                             self.Ci) if self.dual else None
        self._riders = (cell, pix)  # kept alive until the call returns
        return ctypes.byref(cell), (ctypes.byref(pix) if pix is not None else None)

    riders = True  # bucketed step_overlapped: pass-through halves ride the index launches (False: k_dense copies)

    def copy_riders_ok(self, bev, img):
        """The riders' shape rule (16-byte rows and pieces), else the pass-through halves take shpl_pull_dense."""
        esz = self.bv_fused.element_size()
        return self.riders and all((c * esz) % 16 == 0 for c in (self.Cb, self.Ci)) and all(
            t.data_ptr() % 16 == 0 for t in (bev, img, self.bv_fused) + ((self.img_fused,) if self.dual else ()))

    def _pass_copies(self, bev, img, which=("cell", "pixel")):
        """The forward's pass-through halves alone (shpl_pull_dense over no pooled channels): bv_fused[..., :Cb]
        = bev, img_fused[..., :Ci] = img; they need no index."""
        st = L.stream_of(self.dev)
        dt = L.dtype_code(self.bv_fused)
        if "cell" in which:
            L.check(self._lib.shpl_pull_dense(L.BY_CELL, dt, self.csr.ref(), None, 0, 0, 0, L.ptr(bev), self.Cb, 0,
                                              self.Cb, L.OUT_CONCAT, L.ptr(self.bv_fused), self.Cb + self.Ci, st),
                    "shpl_pull_dense")
        if self.dual and "pixel" in which:
            L.check(self._lib.shpl_pull_dense(L.BY_PIXEL, dt, self.pcsr.ref(), None, 0, 0, 0, L.ptr(img), self.Ci, 0,
                                              self.Ci, L.OUT_CONCAT, L.ptr(self.img_fused), self.Ci + self.Cb, st),
                    "shpl_pull_dense")

    def _pooled_descs(self, bev, img, which=("cell", "pixel")):
        """The forward pair's pooled halves (SHPL_OUT_POOL into the output rows' pooled columns)."""
        dt = L.dtype_code(self.bv_fused)
        esz = self.bv_fused.element_size()
        cell = pix = None
        if "cell" in which:
            cell = L.pull_desc(dt, img, self.Ci, 0, self.Ci, None, 0, 0, 0, L.OUT_POOL, self.bv_fused,
                               self.Cb + self.Ci)
            cell.out += self.Cb * esz
        if self.dual and "pixel" in which:
            pix = L.pull_desc(dt, bev, self.Cb, 0, self.Cb, None, 0, 0, 0, L.OUT_POOL, self.img_fused,
                              self.Ci + self.Cb)
            pix.out += self.Ci * esz
        return cell, pix

    def layer_sparse(self, bev, img, which=("cell", "pixel")):
        """Pooled rows, after layer_dense and build_csr (with buckets: the pass-through halves and
        then both pooled halves in one launch)."""
        if self.buckets:
            self._pass_copies(bev, img, which)
            self._pull_pair(*self._pooled_descs(bev, img, which))
            return
        if self.split:
            self._pooled_half(img)
            return
        if "cell" in which:
            self._sparse(self._concat_args(self.csr, L.BY_CELL, img, self.Ci, bev, self.Cb, self.bv_fused))
        if self.dual and "pixel" in which:
            self._sparse(self._concat_args(self.pcsr, L.BY_PIXEL, bev, self.Cb, img, self.Ci, self.img_fused))

    def layer(self, bev, img):
        """bv_fused = [bev || pool(img)] (+ img_fused = [img || trans(bev)] if dual)."""
        self.layer_dense(bev, img)
        self.layer_sparse(bev, img)

    def step(self, points, voxels, point_offsets, P, bev, img, mval=None):
        self.build_index(points, voxels, point_offsets, P, mval)
        self.build_csr()
        self.layer(bev, img)

    def _pooled_half(self, img):
        """split: bv_fused[..., Cb:] = pool(img), every row written once (zeros where no entry lands): the
        row-keyed pull over the cell CSR's key ranges (SHPL_OUT_POOL into the pooled columns)."""
        esz = self.bv_fused.element_size()
        out = ctypes.c_void_p(self.bv_fused.data_ptr() + self.Cb * esz)
        fn = self._lib.shpl_pull_once if self.SPLIT_ONCE else self._lib.shpl_pull
        L.check(fn(L.BY_CELL, L.dtype_code(self.bv_fused), self.csr.ref(), L.ptr(img), self.Ci, 0,
                   self.Ci, None, 0, 0, 0, L.OUT_POOL, out, self.Cb + self.Ci, L.stream_of(self.dev)), "shpl_pull")

    # split: the pooled half after the copy instead of beside it -- each alone at its own rate rather than
    # the two sharing HBM, and the step capturable in a graph (the chain only has to finish under the copy,
    # no stream priority needed): 1.345 vs 1.36 (graph) / 1.385 ms (eager) overlapped at config 6
    # (profiles/r05_c6segg_ab.log)
    SPLIT_SERIAL = True

    def step_split(self, points, voxels, point_offsets, P, bev, img, side, chain, events=None):
        """split: the pass-through copy on `side`, the index chain and then the pooled half on `chain` (a
        high-priority stream, so its latency-bound workgroups are dispatched ahead of the copy's); neither
        waits for the other (disjoint columns of bv_fused). events: [copy start, copy end, chain start, end].
        chain None: the chain runs on the current stream itself (a caller running on a high-priority stream),
        so that one step's chain follows the previous one's with no cross-stream hop; only the copy forks."""
        main = torch.cuda.current_stream(self.dev)
        side.wait_stream(main)
        if chain is None:
            chain = main
        else:
            chain.wait_stream(main)
        # the chain is issued (and, in a captured graph, its nodes created) first: its first launch is
        # dispatched before the copy's workgroups fill the chip
        with torch.cuda.stream(chain):
            if events:
                events[2].record(chain)
            self.build_index(points, voxels, point_offsets, P)
            self.build_csr(("cell",))
            if not self.SPLIT_SERIAL:
                self._pooled_half(img)
                if events:
                    events[3].record(chain)
        with torch.cuda.stream(side):
            if events:
                events[0].record(side)
            self._pass_copies(bev, img, ("cell",))
            if events:
                events[1].record(side)
        if self.SPLIT_SERIAL:
            with torch.cuda.stream(chain):
                chain.wait_stream(side)
                self._pooled_half(img)
                if events:
                    events[3].record(chain)
        main.wait_stream(side)
        if chain is not main:
            main.wait_stream(chain)

    def step_overlapped(self, points, voxels, point_offsets, P, bev, img, side, mval=None, events=None,
                        side2=None):
        """Same result as step(): the streaming half runs on `side` while the
        current stream builds M and its CSR; the sparse half then waits for it.
        Dual layers with `side2`: the pixel-keyed CSR and pull run on side2,
        beside the cell-keyed ones (they share only M).
        `events` (4 timing events) bracket the dense and the sparse launches."""
        if self.buckets:
            # one stream: index + buckets with the pass-through halves riding its two launches, both CSRs
            # (1 launch), both pooled halves (1 launch). (The copies on `side` beside the index chain instead
            # cost 20-30 us of cross-queue waits per graph replay at config 3: profiles/r03_bpull_ab.log.)
            main = torch.cuda.current_stream(self.dev)
            if events:  # no streaming half of its own: the forward bracket [2, 3) is the whole forward
                for e in events[:3]:
                    e.record(main)
            riders = self.copy_riders_ok(bev, img)
            if not riders:
                self._pass_copies(bev, img)
            self.build_index(points, voxels, point_offsets, P, mval, pass_copies=(bev, img) if riders else None)
            self.build_csr()
            self._pull_pair(*self._pooled_descs(bev, img))
            if events:
                events[3].record(main)
            return
        main = torch.cuda.current_stream(self.dev)
        side.wait_stream(main)            # inputs / previous step done
        split = self.dual and side2 is not None
        # dual layers: the cell-keyed sparse pass needs only bv_fused's stream, so it runs
        # beside img_fused's stream (the gathers overlap the second dense pass)
        cell_streamed = torch.cuda.Event() if split and not self.rows and self.interleave else None
        with torch.cuda.stream(side):
            if events:
                events[0].record(side)
            self.layer_dense(bev, img, ("cell",))
            if cell_streamed is not None:
                cell_streamed.record(side)
            self.layer_dense(bev, img, ("pixel",))
            if events:
                events[1].record(side)
        self.build_index(points, voxels, point_offsets, P, mval)
        if split:
            side2.wait_stream(main)       # M built
            with torch.cuda.stream(side2):
                self.build_csr(("pixel",))
                side2.wait_stream(side)
                self.layer_sparse(bev, img, ("pixel",))
        self.build_csr(("cell",) if split else ("cell", "pixel"))
        if cell_streamed is not None:
            main.wait_event(cell_streamed)  # the cell-keyed sparse pass overwrites rows bv_fused's stream wrote
        else:
            main.wait_stream(side)        # sparse overwrites rows the dense pass wrote
        if events:
            events[2].record(main)
        self.layer_sparse(bev, img, ("cell",) if split else ("cell", "pixel"))
        if split:
            main.wait_stream(side2)
        main.wait_stream(side)
        if events:
            events[3].record(main)

    def backward(self, g_bv, g_img, d_bev, d_img, side2=None):
        """TF gradient of the dual layer with the concat split and add_n fused:
        d_bev = g_bv[..., :Cb] + M^T-pull of g_img[..., Ci:]
        d_img = g_img[..., :Ci] + scatter of M-pulled g_bv[..., Cb:].
        With the builder's identity columns the forward entry lists already are
        in the gradients' TF order (ORDER_COL_ENTRY == ORDER_ENTRY / COL_ROW).
        side2: the d_img pull runs there, beside the d_bev pull."""
        assert self.dual
        main = torch.cuda.current_stream(self.dev)
        w = self.Cb + self.Ci
        dt = L.dtype_code(d_bev)
        if self.buckets:  # both gradient pulls, one launch, current stream
            self._pull_pair(L.pull_desc(dt, g_img, w, self.Ci, self.Cb, g_bv, w, 0, self.Cb, L.OUT_ADD, d_bev,
                                        self.Cb),
                            L.pull_desc(dt, g_bv, w, self.Cb, self.Ci, g_img, w, 0, self.Ci, L.OUT_ADD, d_img,
                                        self.Ci))
            return
        cell = (L.BY_CELL, dt, self.csr.ref(), L.ptr(g_img), w, self.Ci, self.Cb, L.ptr(g_bv), w, 0, self.Cb,
                L.OUT_ADD, L.ptr(d_bev), self.Cb)
        pix = (L.BY_PIXEL, dt, self.pcsr.ref(), L.ptr(g_bv), w, self.Cb, self.Ci, L.ptr(g_img), w, 0, self.Ci,
               L.OUT_ADD, L.ptr(d_img), self.Ci)
        pst = side2 if side2 is not None else main
        if side2 is not None:
            side2.wait_stream(main)       # forward done
        L.check(self._lib.shpl_pull(*cell, L.stream_of(self.dev)), "shpl_pull")
        with torch.cuda.stream(pst):
            if not self.rows:
                L.check(self._lib.shpl_pull_dense(*pix, L.stream_of(self.dev)), "shpl_pull_dense")
            self._sparse(pix)
        if side2 is not None:
            main.wait_stream(side2)

    def check(self):
        """Raise if a step since the last check set a bit of the device error word (one device->host read:
        call it outside timed or captured regions). The steps never read it themselves. SHPL_EBIT_BARRIER (the
        one-launch index build gave up at a frame barrier, or found its words not zeroed) raises RuntimeError
        after the word and the barrier words are reset, so the next step can run; an input bit raises
        ShplMap.check's InvalidArgumentError."""
        bits = int(self.err.item()) & 0xFFFFFFFF
        if not bits:
            return
        self.err.zero_()
        if bits & L.EBIT_BARRIER and self.buckets:
            L.bucket_workspace_reset(self.B, self.bkt_ws, self.dev)
        raise_for_bits(bits)

    def map(self):
        """The current M as a ShplMap (for tests)."""
        return ShplMap(self.cell, None, self.val, self.pix, self.N, self.n_cells, self.n_pix, self.N,
                       self.dev, frame_off=self.frame_off, frame_nnz=self.frame_nnz, n_frames=self.B,
                       err=self.err)


def stack_frames(frames, device):
    """Upload a list of synth.Frame to the device as one batch."""
    pts = np.concatenate([f.points for f in frames], axis=0)
    vox = np.concatenate([f.voxel_indices for f in frames], axis=0)
    off = np.zeros(len(frames) + 1, dtype=np.int64)
    off[1:] = np.cumsum([f.points.shape[0] for f in frames])
    P = np.stack([f.P.reshape(12) for f in frames])
    t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(device)  # noqa: E731
    return (t(pts, torch.float64), t(vox, torch.int64), t(off, torch.int64), t(P, torch.float64),
            int(max(f.points.shape[0] for f in frames)), int(pts.shape[0]))


class FramePipeline(FusedPipeline):
    """The whole per-frame SHPL path from raw camera-frame point clouds:
    shpl_bev_slices (BevSlices.generate_bev(output_indices=True), bev_slices.py:33-156)
    -> shpl_build_index on its voxel points (kitti_dataset.py:374-379)
    -> destination-sorted M -> fused layer. bv_size is the BEV map size (nz, nx)."""

    def __init__(self, n_frames, total_points, im_size, area_extents, voxel_size, height_lo, height_hi,
                 num_slices, stride, c_bev, c_img, dtype=torch.float32, device="cuda", dual=False, maps=True,
                 max_points_per_frame=None):
        from . import bev as _bev
        nx, nz = _bev.grid_divisions(area_extents, voxel_size)
        # a frame holds at most as many voxels as points (capacity layout)
        maxp = total_points if max_points_per_frame is None else max_points_per_frame
        super().__init__(n_frames, maxp, total_points, im_size, (nz, nx), stride, c_bev, c_img,
                         dtype=dtype, device=device, dual=dual, live=True)
        self.bev_args = (area_extents, voxel_size, height_lo, height_hi, num_slices)
        self.maps = maps
        import ctypes
        nb = ctypes.c_size_t()
        L.check(self._lib.shpl_bev_workspace_bytes(self.N, int(num_slices), ctypes.byref(nb)),
                "shpl_bev_workspace_bytes")
        self.bev_ws = L.workspace(nb.value, self.dev)
        self.bev = None
        self._velo_ws = None

    # velo_step with a side stream: where the BEV maps are written (shpl_bev_maps) -- "chain": on the
    # index chain after the CSR, beside the end of the streaming pass (step 2.66-2.67 ms); "stream": on the
    # side stream after the streaming pass (2.68-2.69 ms; profiles/r03_frames_maps_ab.log)
    maps_after = "chain"
    # the form of the BEV maps the steps write: "f64" -- the reference's height / density maps
    # (BevSlices.generate_bev, [F,S,nz,nx] + [F,nz,nx] f64); "bev_input" -- the network's BEV input as its
    # tf.float32 placeholder receives it, np.dstack((*height_maps, density_map)) (kitti_dataset.py:368) rounded
    # to f32 once ([F,nz,nx,S+1]; shpl_bev_input): half the bytes, the layout the BEV extractor reads
    maps_form = "f64"
    # where velo_step starts the streaming half: "start" (beside the whole index chain), or after the
    # chain's "velo" / "bev" / "csr" stage (the chain then runs with the chip to itself until there)
    dense_after = "start"
    DENSE_AFTER, MAPS_AFTER, MAPS_FORMS = ("start", "velo", "bev", "csr"), ("stream", "chain"), ("f64", "bev_input")

    def build_bev(self, points, point_offsets, planes, point_counts=None, maps=None):
        from . import bev as _bev
        want = self.maps if maps is None else maps
        self.bev = _bev.bev_slices_batch(points, point_offsets, planes, *self.bev_args,
                                         maps=want and self.maps_form == "f64", ws=self.bev_ws,
                                         point_counts=point_counts)
        if want and self.maps_form == "bev_input":
            self.bev.write_bev_input(self._input_buffer())
        return self.bev

    def _input_buffer(self):
        """The step's BEV input tensor [F,nz,nx,S+1] f32 (maps_form "bev_input"), allocated once."""
        if getattr(self, "_bev_input", None) is None:
            from . import bev as _bev
            area, vs, _, _, S = self.bev_args
            nx, nz = _bev.grid_divisions(area, vs)
            self._bev_input = torch.empty((self.B, nz, nx, int(S) + 1), dtype=torch.float32, device=self.dev)
        return self._bev_input

    def _write_maps(self, b):
        if self.maps_form == "bev_input":
            b.write_bev_input(self._input_buffer())
        else:
            b.write_maps(*self._map_buffers(), zero=True)

    def _map_buffers(self):
        """The step's height / density maps, allocated once (velo_step writes them off the chain)."""
        if getattr(self, "_maps", None) is None:
            from . import bev as _bev
            area, vs, _, _, S = self.bev_args
            nx, nz = _bev.grid_divisions(area, vs)
            f64 = dict(dtype=torch.float64, device=self.dev)
            self._maps = (torch.empty((self.B, int(S), nz, nx), **f64), torch.empty((self.B, nz, nx), **f64))
        return self._maps

    def frame_step(self, points, point_offsets, planes, P, bev_feat, img_feat, point_counts=None):
        b = self.build_bev(points, point_offsets, planes, point_counts)
        self.build_index(b.pts_in_voxel, b.voxel_indices, point_offsets, P, point_counts=b.frame_nvox)
        self.build_csr()
        self.layer(bev_feat, img_feat)

    def velo_step(self, frames, bev_feat, img_feat, side=None, events=None):
        """Raw KITTI scans (kitti.KittiFrames) -> camera-frame clouds (shpl_velo_to_cam)
        -> BEV slices -> M -> fused layer, all on the device (kitti_dataset.py:285-379).
        side: a stream for the layer's streaming half (it needs no index), run beside
        the index chain. events: 9 timing events (dense start/end on `side`; then
        velo, bev, index, csr boundaries, sparse start/end on the current stream)."""
        if self.dense_after not in self.DENSE_AFTER:
            raise ValueError(f"dense_after must be one of {self.DENSE_AFTER}, not {self.dense_after!r}")
        if self.maps_after not in self.MAPS_AFTER:
            raise ValueError(f"maps_after must be one of {self.MAPS_AFTER}, not {self.maps_after!r}")
        if self.maps_form not in self.MAPS_FORMS:
            raise ValueError(f"maps_form must be one of {self.MAPS_FORMS}, not {self.maps_form!r}")
        if side is not None:
            # the 1.7 GB of f64 maps (64 frames) are written on `side` after the streaming pass, from the
            # voxelizer's sorted words (shpl_bev_maps): off the index chain, and streaming after the
            # stream instead of beside it
            main = torch.cuda.current_stream(self.dev)
            dense_done, bev_done = torch.cuda.Event(), torch.cuda.Event()

            def dense():  # the streaming half on `side`, after what `main` has issued so far
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    if events:
                        events[0].record(side)
                    self.layer_dense(bev_feat, img_feat)
                    dense_done.record(side)
                    if events:
                        events[1].record(side)

            at = self.dense_after
            if at == "start":
                dense()
            if events:
                events[2].record(main)
            self._velo(frames)
            if events:
                events[3].record(main)
            if at == "velo":
                dense()
            b = self.build_bev(self.velo.points, frames.point_offsets, frames.planes, self.velo.counts,
                               maps=False)
            bev_done.record(main)
            if at == "bev":
                dense()
            if self.maps and self.maps_after == "stream":
                side.wait_event(bev_done)
                with torch.cuda.stream(side):
                    self._write_maps(b)
            if events:
                events[4].record(main)
            self.build_index(b.pts_in_voxel, b.voxel_indices, frames.point_offsets, frames.P2,
                             point_counts=b.frame_nvox)
            if events:
                events[5].record(main)
            self.build_csr()
            if events:
                events[6].record(main)
            if at == "csr":
                dense()
            if self.maps and self.maps_after == "chain":
                self._write_maps(b)
            main.wait_event(dense_done)  # the sparse pass overwrites rows the streaming pass wrote
            if events:
                events[7].record(main)
            self.layer_sparse(bev_feat, img_feat)
            if events:
                events[8].record(main)
            main.wait_stream(side)  # the maps
            return
        self._velo(frames)
        self.frame_step(self.velo.points, frames.point_offsets, frames.planes, frames.P2, bev_feat, img_feat,
                        point_counts=self.velo.counts)

    def _velo(self, frames):
        if self._velo_ws is None:
            import ctypes
            nb = ctypes.c_size_t()
            L.check(self._lib.shpl_velo_workspace_bytes(frames.n_frames, frames.max_points, ctypes.byref(nb)),
                    "shpl_velo_workspace_bytes")
            self._velo_ws = L.workspace(nb.value, self.dev)
            self._velo_pts = torch.empty((max(self.N, 1), 3), dtype=torch.float64, device=self.dev)
        self.velo = frames.point_clouds(ws=self._velo_ws, out=self._velo_pts)
