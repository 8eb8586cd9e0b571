"""Tuning sweep of the pull kernel on the GPU box: times compile-time variants
of libshpl (built by `python scripts/pull_sweep.py --build`) on the bench
workload (64 config-2 frames). Also calibrates the box's copy bandwidth."""
import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "sparse_pooling_amd", "variants")

VARIANTS = {
    "base": [],
    "d16k": ["-DSHPL_DENSE_BLOCKS=16384"],
    "d64k": ["-DSHPL_DENSE_BLOCKS=65536"],
    "dfull": ["-DSHPL_DENSE_BLOCKS=2147483647"],
    "dfull_u2": ["-DSHPL_DENSE_BLOCKS=2147483647", "-DSHPL_PULL_U=2"],
    "dfull_u1": ["-DSHPL_DENSE_BLOCKS=2147483647", "-DSHPL_PULL_U=1"],
    "t2k": ["-DSHPL_DENSE_TILED=1"],
    "t16k": ["-DSHPL_DENSE_TILED=1", "-DSHPL_DENSE_BLOCKS=16384"],
    "tfull": ["-DSHPL_DENSE_TILED=1", "-DSHPL_DENSE_BLOCKS=2147483647"],
    "tfull_u8": ["-DSHPL_DENSE_TILED=1", "-DSHPL_DENSE_BLOCKS=2147483647", "-DSHPL_PULL_U=8"],
    "t16k_u8": ["-DSHPL_DENSE_TILED=1", "-DSHPL_DENSE_BLOCKS=16384", "-DSHPL_PULL_U=8"],
    "dfull_s8k": ["-DSHPL_DENSE_BLOCKS=2147483647", "-DSHPL_SPARSE_BLOCKS=8192"],
    "dfull_sfull": ["-DSHPL_DENSE_BLOCKS=2147483647", "-DSHPL_SPARSE_BLOCKS=2147483647"],
}


def build():
    from sparse_pooling_amd import build as b
    b.build()
    os.makedirs(VDIR, exist_ok=True)
    objs = [o for o in glob.glob(os.path.join(ROOT, "sparse_pooling_amd", "csrc", "build", "*.o"))
            if not o.endswith("shpl_pull.o")]
    for name, defs in VARIANTS.items():
        o = os.path.join(VDIR, f"pull_{name}.o")
        subprocess.run([b.HIPCC, *b.FLAGS, *defs, "-c", os.path.join(b.CSRC, "shpl_pull.hip"), "-o", o],
                       check=True)
        subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, o, "-o",
                        os.path.join(VDIR, f"libshpl_{name}.so")], check=True)
        print("built", name)


def run(reps):
    import torch
    from sparse_pooling_amd import _lib as L, pipeline, synth
    spec = synth.CONFIGS[2]
    F = 64
    dev = torch.device("cuda", 0)
    frames = [synth.make_frame(spec, seed=f, n_outside=200) for f in range(F)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
    pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                device=dev)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = torch.randn((F, Hb, Wb, spec.c_bev), device=dev)
    img = torch.randn((F, Hi, Wi, spec.c_img), device=dev)
    pl.step(pts, vox, off, P, bev, img)
    torch.cuda.synchronize()
    nnz = int(pl.frame_nnz.sum().item())
    u_src = int(torch.unique(pl.pix[pl.pix >= 0]).numel())
    import bench
    nbytes = bench.layer_bytes(spec, nnz, u_src, F)
    ref = pl.bv_fused.clone()
    res = {}

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    # calibration: device-to-device copy of the same byte count class
    src = torch.empty(nbytes // 2 // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    ms = timeit(lambda: dst.copy_(src))
    res["torch_copy"] = {"ms": ms, "GBps": 2 * src.numel() * 4 / ms / 1e6}
    cal = ctypes.CDLL(os.path.join(VDIR, "libcalib.so"))
    st0 = L.stream_of(dev)
    n16 = src.numel() // 4
    for unroll in (1, 2, 4):
        for nt in (0, 1):
            for grid in (0, 2048, 16384):
                ms = timeit(lambda: cal.calib_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                                   ctypes.c_uint64(n16), unroll, nt, grid, st0))
                res[f"copy_u{unroll}_nt{nt}_g{grid}"] = round(2 * src.numel() * 4 / ms / 1e6, 1)
    rows = F * Hb * Wb
    for nt in (0, 1):
        for grid in (0, 2048, 16384):
            ms = timeit(lambda: cal.calib_concat_zero(ctypes.c_void_p(bev.data_ptr()), ctypes.c_void_p(pl.bv_fused.data_ptr()),
                                                      ctypes.c_uint32(rows), ctypes.c_uint32(16), ctypes.c_uint32(8),
                                                      nt, grid, st0))
            res[f"concat_zero_nt{nt}_g{grid}"] = {"ms": round(ms, 4), "GBps": round(3 * rows * 128 / ms / 1e6, 1)}
    ms = timeit(lambda: cal.calib_zero(ctypes.c_void_p(pl.bv_fused.data_ptr()), ctypes.c_uint64(rows * 16), 0, st0))
    res["zero_fill"] = round(rows * 256 / ms / 1e6, 1)
    print({k: v for k, v in res.items()}, flush=True)
    # empty CSR: dense role alone (zeros + pass-through)
    empty = L.Csr(pl.n_cells, 1, dev, with_col=False)
    empty.ent_dst.fill_(-1)
    for name in VARIANTS:
        path = os.path.join(VDIR, f"libshpl_{name}.so")
        if not os.path.exists(path):
            continue
        lib = ctypes.CDLL(path)
        lib.shpl_pull.restype = ctypes.c_int
        lib.shpl_pull.argtypes = L.lib().shpl_pull.argtypes
        st = L.stream_of(dev)

        def call(c=pl.csr):
            rc = lib.shpl_pull(L.BY_CELL, L.F32, c.ref(), L.ptr(img), 32, 0, 32, L.ptr(bev), 32, 0, 32,
                               L.OUT_CONCAT, L.ptr(pl.bv_fused), 64, st)
            assert rc == 0
        ms = timeit(call)
        ok = bool(torch.equal(pl.bv_fused, ref))
        ms_dense = timeit(lambda: call(empty))
        res[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1), "exact": ok,
                     "dense_only_ms": round(ms_dense, 4)}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(a.reps)
