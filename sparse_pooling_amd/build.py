"""Build libshpl.so (the HIP kernels + C ABI) in-tree for gfx950.

    python -m sparse_pooling_amd.build

hipcc cross-compiles without a GPU; the .so is git-ignored but travels to
the GPU box with the gpurun snapshot.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libshpl.so")
OBJ = os.path.join(HERE, "csrc", "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function"]


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
    deps = [src, *glob.glob(os.path.join(CSRC, "*.h")),
            os.path.join(os.path.dirname(HERE), "include", "shpl.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    subprocess.run([HIPCC, *FLAGS, "-c", src, "-o", obj], check=True)
    return obj


def build(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(o) for o in objs):
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", OUT],
                       check=True)
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
