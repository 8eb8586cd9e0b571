"""Write-rate calibration for config 6's split layer (not part of the library): the pass-through copy of
64 x 35,200 rows of 1 KB (256 f32) by shpl_pull_dense (no pooled channels)
  half  -- into the first half of 2 KB output rows (bv_fused's layout: the split step's copy)
  cont  -- into contiguous 1 KB rows (the same bytes, no gaps)
  full  -- the concat's whole 2 KB rows (pass-through + pooled zeros: what a pass writing each row once
           would stream)
and the pooled zeros alone into the second halves (zhalf). HIP events around 20 launches each."""
import ctypes
import torch
from sparse_pooling_amd import _lib as L

dev = torch.device("cuda:0")
R, C = 64 * 35200, 256
bev = torch.randn(R, C, device=dev)
out = torch.empty(R, 2 * C, device=dev)
cont = torch.empty(R, C, device=dev)
lib = L.lib()


def dense(src_c_pool, pass_, out_ptr, out_stride, c_pass):
    c = L.ShplCsr()
    c.n_keys = R
    L.check(lib.shpl_pull_dense(L.BY_CELL, L.dtype_code(bev), ctypes.byref(c), L.ptr(bev), C, 0, src_c_pool,
                                L.ptr(pass_) if pass_ is not None else None, C, 0, c_pass,
                                L.OUT_CONCAT if c_pass else L.OUT_POOL, ctypes.c_void_p(out_ptr), out_stride,
                                L.stream_of(dev)), "shpl_pull_dense")


forms = {
    "half": (lambda: dense(0, bev, out.data_ptr(), 2 * C, C), 2 * R * C * 4),
    "cont": (lambda: dense(0, bev, cont.data_ptr(), C, C), 2 * R * C * 4),
    "full": (lambda: dense(C, bev, out.data_ptr(), 2 * C, C), 3 * R * C * 4),
    "zhalf": (lambda: dense(C, None, out.data_ptr() + C * 4, 2 * C, 0), R * C * 4),
}
for name, (fn, nbytes) in list(forms.items()) * 2:
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    print(f"{name:6s} {ms:.4f} ms  {nbytes / 1e9:.2f} GB  {nbytes / ms / 1e6:.0f} GB/s", flush=True)
