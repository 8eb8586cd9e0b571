"""Sweep of k_sparse compile-time variants (run-walk batch WALK, predicated
index loads) on the GPU box: times shpl_pull_sparse alone on the config-2
(64 frames, f32, BEV-cell pull) and config-3 (4 frames, bf16, both
directions) maps, and checks each variant bit-exact against the default
library.  `python scripts/sparse_sweep.py --build` (here), then without
--build on the box."""
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

VARIANTS = {f"w{w}_p{p}": [f"-DSHPL_WALK={w}", f"-DSHPL_WALK_PRED={p}"] for w in (1, 2, 4, 8) for p in (0, 1)}
# (profiles/r01_sparse_sweep.log also holds a timing-only experiment that cut the
# run walk after 2/8/16 entries: c3_pix 9.6/19.0/27.4 us against 38.5 us in full --
# the pixel-keyed pull is bound by the long runs of coarse-stride pixels.)


def build():
    from sparse_pooling_amd import build as b
    b.build()
    os.makedirs(VDIR, exist_ok=True)
    objs = [o for o in glob.glob(os.path.join(ROOT, "sparse_pooling_amd", "csrc", "build", "*.o"))
            if not o.endswith("shpl_pull.o")]
    for name, defs in VARIANTS.items():
        o = os.path.join(VDIR, f"sparse_{name}.o")
        subprocess.run([b.HIPCC, *b.FLAGS, *defs, "-c", os.path.join(b.CSRC, "shpl_pull.hip"), "-o", o],
                       check=True)
        subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, o, "-o",
                        os.path.join(VDIR, f"libshpl_sparse_{name}.so")], check=True)
        print("built", name, flush=True)


def run(reps):
    import torch
    from sparse_pooling_amd import _lib as L, pipeline, synth
    dev = torch.device("cuda", 0)
    cases = []
    for cfg, F, dtype in ((2, 64, torch.float32), (3, 4, torch.bfloat16)):
        spec = synth.CONFIGS[cfg]
        frames = [synth.make_frame(spec, seed=f, n_outside=200) for f in range(F)]
        pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
        pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev,
                                    spec.c_img, dtype=dtype, device=dev, dual=cfg == 3)
        bev = torch.randn((F, pl.Hb, pl.Wb, spec.c_bev), device=dev).to(dtype)
        img = torch.randn((F, pl.Hi, pl.Wi, spec.c_img), device=dev).to(dtype)
        pl.step(pts, vox, off, P, bev, img)
        cases.append((f"c{cfg}_cell", pl, L.BY_CELL, pl.csr, img, spec.c_img, bev, spec.c_bev, pl.bv_fused))
        if cfg == 3:
            cases.append((f"c{cfg}_pix", pl, L.BY_PIXEL, pl.pcsr, bev, spec.c_bev, img, spec.c_img, pl.img_fused))
    torch.cuda.synchronize()

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

    refs = {c[0]: c[8].clone() for c in cases}
    res = {}
    for name in VARIANTS:
        path = os.path.join(VDIR, f"libshpl_sparse_{name}.so")
        lib = ctypes.CDLL(path)
        lib.shpl_pull_sparse.restype = ctypes.c_int
        lib.shpl_pull_sparse.argtypes = L.lib().shpl_pull_sparse.argtypes
        st = L.stream_of(dev)
        row = {}
        for cname, pl, direction, csr, src, cs, pas, cp, out in cases:
            def call():
                rc = lib.shpl_pull_sparse(direction, L.dtype_code(out), csr.ref(), L.ptr(src), cs, 0, cs,
                                          L.ptr(pas), cp, 0, cp, L.OUT_CONCAT, L.ptr(out), cs + cp, st)
                assert rc == 0
            ms = timeit(call)
            row[cname] = {"us": round(1e3 * ms, 1), "exact": bool(torch.equal(out, refs[cname]))}
            # run-length profile of this map (first variant only)
            if name == next(iter(VARIANTS)):
                d = csr.ent_dst[csr.ent_dst >= 0]
                _, counts = torch.unique_consecutive(d, return_counts=True)
                row[cname]["runs"] = {"n": int(counts.numel()), "max": int(counts.max()),
                                      "gt8": int((counts > 8).sum()), "gt16": int((counts > 16).sum())}
        res[name] = row
        print(name, row, flush=True)
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
