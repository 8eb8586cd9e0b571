"""ctypes binding of libshpl.so (include/shpl.h).

The product path has no fallback: if the HIP library is missing or cannot be
loaded, every SHPL op raises ``ShplLibraryError``. Tensors cross the C ABI as
raw device pointers plus the current HIP stream of the calling thread.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# SHPL_LIB: an alternative build of the same sources (A/B measurements of compile-time variants)
LIB_PATH = os.environ.get("SHPL_LIB") or os.path.join(_HERE, "libshpl.so")

# enums of include/shpl.h
OK, ERR_BAD_SHAPE, ERR_INDEX_OOB, ERR_HIP, ERR_WORKSPACE, ERR_ARG = range(6)
EBIT_ROW, EBIT_COL, EBIT_PIXEL, EBIT_VALUES, EBIT_CAPACITY, EBIT_BARRIER = 1, 2, 4, 8, 16, 32
F32, BF16, F64 = 0, 1, 2
I32, I64 = 0, 1
BY_CELL, BY_PIXEL = 0, 1
ORDER_ENTRY, ORDER_COL_ROW, ORDER_COL_ENTRY = 0, 1, 2
OUT_POOL, OUT_CONCAT, OUT_ADD = 0, 1, 2
ACT_NONE, ACT_RELU = 0, 1
CSR_AUTO, CSR_FRAME, CSR_SEGMENT, CSR_RANGE = 0, 1, 2, 3
CSR_IDENTITY_COLS = 1
CSR_MAX_HEAD = 32

_lib = None


class ShplLibraryError(RuntimeError):
    pass


LIVE_MAX_FRAMES = 1024  # SHPL_LIVE_MAX_FRAMES


class ShplCsr(ctypes.Structure):
    """struct shpl_csr of include/shpl.h (device pointers + sizes)."""
    _fields_ = [("ent_dst", ctypes.c_void_p), ("ent_src", ctypes.c_void_p),
                ("ent_val", ctypes.c_void_p), ("ent_col", ctypes.c_void_p),
                ("n_keys", ctypes.c_int64), ("nnz_cap", ctypes.c_int64), ("key_range", ctypes.c_void_p),
                ("frame_off", ctypes.c_void_p), ("frame_nnz", ctypes.c_void_p), ("n_frames", ctypes.c_int64),
                ("flags", ctypes.c_int64), ("heads", ctypes.c_void_p), ("head_k", ctypes.c_int64)]


class Csr:
    """Device buffers of one destination-sorted entry list (owned tensors + the ABI struct)."""

    def __init__(self, n_keys, nnz_cap, device, with_col, key_range=False, identity_cols=False, head_k=0):
        """key_range: also keep the (first, end) entry of every destination
        (shpl_csr.key_range): shpl_pull then runs its one-launch row-keyed form.
        identity_cols: a pixel-keyed CSR of shpl_build_csr_buckets without ent_col (SHPL_CSR_IDENTITY_COLS).
        head_k: run heads of that many entries per destination (shpl_csr.heads; shpl_build_csr_buckets)."""
        i32 = dict(dtype=torch.int32, device=device)
        cap = max(int(nnz_cap), 1)
        self.n_keys, self.nnz_cap = int(n_keys), int(nnz_cap)
        self.ent_dst = torch.empty(cap, **i32)
        self.ent_src = torch.empty(cap, **i32)
        self.ent_val = torch.empty(cap, dtype=torch.float32, device=device)
        self.ent_col = torch.empty(cap, **i32) if with_col else None
        self.key_range = torch.empty((max(self.n_keys, 1), 2), **i32) if key_range else None
        self.ws = workspace(csr_ws_bytes(self.n_keys, self.nnz_cap), device)
        self.struct = ShplCsr(self.ent_dst.data_ptr(), self.ent_src.data_ptr(), self.ent_val.data_ptr(),
                              self.ent_col.data_ptr() if with_col else None, self.n_keys, self.nnz_cap,
                              self.key_range.data_ptr() if key_range else None)
        self.struct.flags = CSR_IDENTITY_COLS if identity_cols else 0
        self.heads = None
        if head_k:
            assert key_range and 1 <= head_k <= CSR_MAX_HEAD
            self.heads = torch.empty((max(self.n_keys, 1), int(head_k), 2), **i32)
            self.struct.heads, self.struct.head_k = self.heads.data_ptr(), int(head_k)

    def live_frames(self, frame_off, frame_nnz):
        """Hand the sparse pass the frame layout the CSR was built with (device i64 [F+1] / [F],
        kept alive here): it then walks only the live entries of each frame's capacity."""
        if frame_nnz is None or frame_nnz.numel() > LIVE_MAX_FRAMES:
            self._frames = None
            self.struct.frame_off, self.struct.frame_nnz, self.struct.n_frames = None, None, 0
            return self
        assert frame_off.dtype == torch.int64 and frame_nnz.dtype == torch.int64
        assert frame_off.numel() == frame_nnz.numel() + 1
        self._frames = (frame_off, frame_nnz)
        self.struct.frame_off, self.struct.frame_nnz = frame_off.data_ptr(), frame_nnz.data_ptr()
        self.struct.n_frames = int(frame_nnz.numel())
        return self

    def ref(self):
        return ctypes.byref(self.struct)


class ShplBuckets(ctypes.Structure):
    """struct shpl_buckets of include/shpl.h."""
    _fields_ = [("n_frames", ctypes.c_int), ("max_points_per_frame", ctypes.c_int64), ("nnz_cap", ctypes.c_int64),
                ("cells_per_frame", ctypes.c_int64), ("pix_per_frame", ctypes.c_int64),
                ("frame_off", ctypes.c_void_p), ("frame_nnz", ctypes.c_void_p), ("cell", ctypes.c_void_p),
                ("pix", ctypes.c_void_p), ("val", ctypes.c_void_p), ("ws", ctypes.c_void_p),
                ("ws_bytes", ctypes.c_size_t), ("err", ctypes.c_void_p)]


class ShplPullDesc(ctypes.Structure):
    """struct shpl_pull_desc of include/shpl.h: shpl_pull's arguments after its csr (shpl_pull_pair)."""
    _fields_ = [("dtype", ctypes.c_int), ("src", ctypes.c_void_p), ("src_stride", ctypes.c_int64),
                ("src_off", ctypes.c_int64), ("c_pool", ctypes.c_int64), ("pass_", ctypes.c_void_p),
                ("pass_stride", ctypes.c_int64), ("pass_off", ctypes.c_int64), ("c_pass", ctypes.c_int64),
                ("mode", ctypes.c_int), ("out", ctypes.c_void_p), ("out_stride", ctypes.c_int64)]


class ShplPassCopy(ctypes.Structure):
    """struct shpl_pass_copy of include/shpl.h (a rider of shpl_build_index_buckets)."""
    _fields_ = [("dtype", ctypes.c_int), ("src", ctypes.c_void_p), ("src_stride", ctypes.c_int64),
                ("out", ctypes.c_void_p), ("out_stride", ctypes.c_int64), ("channels", ctypes.c_int64)]


def pull_desc(dtype, src, src_stride, src_off, c_pool, pass_, pass_stride, pass_off, c_pass, mode, out, out_stride):
    """A ShplPullDesc from tensors (the same argument order as shpl_pull after its csr)."""
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    return ShplPullDesc(dtype, p(src), src_stride, src_off, c_pool, p(pass_), pass_stride, pass_off, c_pass, mode,
                        p(out), out_stride)


def _declare(lib):
    p, i32, i64, d, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_size_t
    psz = ctypes.POINTER(ctypes.c_size_t)
    pull_args = [i32, i32, ctypes.POINTER(ShplCsr), p, i64, i64, i64, p, i64, i64, i64, i32, p, i64, p]
    sig = {
        "shpl_version": (ctypes.c_char_p, []),
        "shpl_status_string": (ctypes.c_char_p, [i32]),
        "shpl_build_index_workspace_bytes": (i32, [i32, i64, psz]),
        "shpl_build_index": (i32, [i32, p, p, i64, p, i32, p, i32, i64, p, d, d, d, d, d, d, p,
                                   p, p, p, p, p, p, p, p, p, sz, p]),
        "shpl_bev_workspace_bytes": (i32, [i64, i32, psz]),
        "shpl_mv3d_workspace_bytes": (i32, [i64, psz]),
        "shpl_mv3d_voxels": (i32, [i32, p, i64, p, i64, p, p, p, p, d, d, i32, p, i64, p, p, p, p, p, p,
                                   sz, p]),
        "shpl_bev_slices": (i32, [i32, p, p, i64, p, i32, p, p, d, i32, p, p, d, d, d, p, p, p, p, p, p,
                                  p, p, sz, p]),
        "shpl_bev_maps": (i32, [i32, p, i64, p, i32, p, p, d, i32, p, p, d, d, d, p, p, p, i32, p, sz, p]),
        "shpl_bev_input": (i32, [i32, p, i64, p, i32, p, p, d, i32, p, p, d, d, d, p, p, p, sz, p]),
        "shpl_velo_workspace_bytes": (i32, [i32, i64, psz]),
        "shpl_velo_to_cam": (i32, [i32, p, i64, p, p, p, p, d, p, p, p, p, p, sz, p]),
        "shpl_gen_index": (i32, [i64, p, i32, p, i32, i64, p, d, d, p, p, i64, p, p, sz, p]),
        "shpl_produce_index": (i32, [i64, p, i32, i64, p, i64, d, d, d, d, d, d, p, p, p, p, p,
                                     p, p, sz, p]),
        "shpl_pack_map": (i32, [i64, p, p, i64, i64, i64, p, i32, i64, i64, i64, i64, i64, i64,
                                p, p, p, p, p, p]),
        "shpl_csr_workspace_bytes": (i32, [i64, i64, psz]),
        "shpl_build_csr": (i32, [i32, i32, i32, p, p, i64, p, p, p, p, ctypes.POINTER(ShplCsr), p, sz,
                                 p]),
        "shpl_build_csr_path": (i32, [i32, i32, i32, i32, p, p, i64, p, p, p, p, ctypes.POINTER(ShplCsr), p,
                                      sz, p]),
        "shpl_bucket_workspace_bytes": (i32, [i32, i64, i64, i64, i64, psz]),
        "shpl_bucket_workspace_reset": (i32, [i32, p, sz, p]),
        "shpl_build_index_buckets": (i32, [i32, p, p, i64, p, i32, p, i32, i64, p, d, d, d, d, d, d, p,
                                           p, p, p, p, p, p, p, sz, i64, p, sz, ctypes.POINTER(ShplPassCopy),
                                           ctypes.POINTER(ShplPassCopy), p]),
        "shpl_build_csr_buckets": (i32, [ctypes.POINTER(ShplBuckets), ctypes.POINTER(ShplCsr),
                                         ctypes.POINTER(ShplCsr), p]),
        "shpl_pull_pair": (i32, [ctypes.POINTER(ShplCsr), ctypes.POINTER(ShplPullDesc), ctypes.POINTER(ShplCsr),
                                 ctypes.POINTER(ShplPullDesc), p]),
        "shpl_pull": (i32, pull_args),
        "shpl_pull_dense": (i32, pull_args),
        "shpl_pull_sparse": (i32, pull_args),
        "shpl_pull_once": (i32, pull_args),
        "shpl_conv3x3_workspace_bytes": (i32, [i32, i32, i64, i64, i64, i64, i64, i64, i32, psz]),
        "shpl_conv3x3": (i32, [i32, i32, i64, i64, p, i64, i64, i64, p, i64, i64, i64,
                               ctypes.POINTER(ShplCsr), p, p, i64, p, p, p, i32, p, i64, p, p, sz, p]),
        "shpl_conv3x3_rows_form": (i32, [i32, i32, i64, i64, p, i64, i64, i64, p, i64, i64, i64,
                                         ctypes.POINTER(ShplCsr), p, p, i64, i32, p, i64, i32,
                                         ctypes.POINTER(ctypes.c_int)]),
        "shpl_batch_norm": (i32, [i32, i64, p, p, i64, i64, p, d, ctypes.c_float, p, p, i32, p, p,
                                  ctypes.c_float, p, p, p, p]),
        "shpl_batch_norm_backward_workspace_bytes": (i32, [i64, i64, psz]),
        "shpl_batch_norm_backward": (i32, [i32, i64, p, p, p, i64, i64, p, p, p, p, i32, i32, p, p, p, p, sz, p]),
        "shpl_conv3x3_dgrad": (i32, [i32, i32, i64, i64, p, i64, i64, p, i64, p, i64, i64, p, i64, p, sz, p]),
        "shpl_conv3x3_dgrad_reuse": (i32, [i32, i32, i64, i64, p, i64, i64, p, i64, p, i64, i64, p, i64, p, sz,
                                           ctypes.POINTER(ShplCsr), p, sz, i32, p]),
        "shpl_conv3x3_wgrad_workspace_bytes": (i32, [i32, i32, i64, i64, i64, i64, i64, i64, psz]),
        "shpl_conv3x3_wgrad": (i32, [i32, i32, i64, i64, p, i64, i64, i64, p, i64, i64, i64,
                                     ctypes.POINTER(ShplCsr), p, p, i64, i64, p, p, sz, p]),
        "shpl_conv3x3_wgrad_reuse": (i32, [i32, i32, i64, i64, p, i64, i64, i64, p, i64, i64, i64,
                                           ctypes.POINTER(ShplCsr), p, p, i64, i64, p, p, sz, p, sz, i32, p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return sig


EXPORTED = None


def lib():
    """Load libshpl.so once; raise loudly if it is absent (no CPU fallback)."""
    global _lib, EXPORTED
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ShplLibraryError(
                f"{LIB_PATH} not found: build it with `python -m sparse_pooling_amd.build` "
                "(the SHPL path has no CPU fallback)")
        try:
            _lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise ShplLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        EXPORTED = sorted(_declare(_lib))
    return _lib


def check(rc, what):
    if rc != OK:
        msg = lib().shpl_status_string(rc).decode()
        raise ShplLibraryError(f"{what} failed: {msg} (status {rc})")


def ptr(t):
    """Device pointer of a tensor (NULL for None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def index_ws_bytes(n_frames, max_points):
    out = ctypes.c_size_t()
    check(lib().shpl_build_index_workspace_bytes(int(n_frames), int(max_points), ctypes.byref(out)),
          "shpl_build_index_workspace_bytes")
    return out.value


def csr_ws_bytes(n_keys, nnz_cap):
    out = ctypes.c_size_t()
    check(lib().shpl_csr_workspace_bytes(int(n_keys), int(nnz_cap), ctypes.byref(out)),
          "shpl_csr_workspace_bytes")
    return out.value


def dtype_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"SHPL features must be float32 or bfloat16, got {t.dtype}")


def bucket_ws_bytes(n_frames, max_points, nnz_cap, cells_per_frame, pix_per_frame):
    out = ctypes.c_size_t()
    check(lib().shpl_bucket_workspace_bytes(int(n_frames), int(max_points), int(nnz_cap), int(cells_per_frame),
                                            int(pix_per_frame), ctypes.byref(out)), "shpl_bucket_workspace_bytes")
    return out.value


def bucket_workspace(n_frames, max_points, nnz_cap, cells_per_frame, pix_per_frame, device):
    """A bucket workspace for shpl_build_index_buckets, ZEROED: its frame barrier words must start at zero
    (include/shpl.h; every call leaves them so, and shpl_bucket_workspace_reset restores them after a
    SHPL_EBIT_BARRIER)."""
    nb = bucket_ws_bytes(n_frames, max_points, nnz_cap, cells_per_frame, pix_per_frame)
    return torch.zeros(max(int(nb), 256), dtype=torch.uint8, device=device)


def bucket_workspace_reset(n_frames, ws, device=None):
    """shpl_bucket_workspace_reset on the current stream."""
    check(lib().shpl_bucket_workspace_reset(int(n_frames), ptr(ws), ws.numel(), stream_of(device)),
          "shpl_bucket_workspace_reset")
