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


def _compile(src, obj_dir=OBJ, extra=()):
    obj = os.path.join(obj_dir, os.path.basename(src).replace(".hip", ".o"))
    deps = [src, *glob.glob(os.path.join(CSRC, "*.h")),
            os.path.join(os.path.dirname(HERE), "include", "shpl.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    subprocess.run([HIPCC, *FLAGS, *extra, "-c", src, "-o", obj], check=True)
    return obj


def build(verbose=False, out=OUT, defines=()):
    """defines: extra -D flags for an A/B variant (with `out` elsewhere, loaded through SHPL_LIB)."""
    obj_dir = OBJ if not defines else os.path.join(OBJ, "variant_" + "_".join(d.replace("=", "") for d in defines))
    os.makedirs(obj_dir, exist_ok=True)
    extra = [f"-D{d}" for d in defines]
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, obj_dir, extra), srcs))
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out],
                       check=True)
    if verbose:
        print("built", out)
    if out == OUT and not defines:
        build_fault(objs, verbose)
    return out


# Test-only library: libshpl.so with shpl_index.hip built with SHPL_IDX1_FAULT=1 (chunk 0 of frame 0 skips its
# frame-barrier arrival, so k_index1's give-up path runs; tests/test_gpu_parity.py loads it by path). Never the
# product library: _lib.LIB_PATH is libshpl.so.
FAULT_OUT = os.path.join(HERE, "libshpl_fault.so")


def build_fault(objs, verbose=False):
    obj_dir = os.path.join(OBJ, "fault")
    os.makedirs(obj_dir, exist_ok=True)
    fault = _compile(os.path.join(CSRC, "shpl_index.hip"), obj_dir, ["-DSHPL_IDX1_FAULT=1"])
    objs = [fault if os.path.basename(o) == "shpl_index.o" else o for o in objs]
    if not os.path.exists(FAULT_OUT) or os.path.getmtime(FAULT_OUT) < max(os.path.getmtime(o) for o in objs):
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", FAULT_OUT], check=True)
    if verbose:
        print("built", FAULT_OUT)
    return FAULT_OUT


if __name__ == "__main__":
    # python -m sparse_pooling_amd.build [OUT.so NAME=VALUE ...]: an A/B variant
    if len(sys.argv) > 2:
        build(verbose=True, out=os.path.abspath(sys.argv[1]), defines=tuple(sys.argv[2:]))
    else:
        build(verbose=True)
    sys.exit(0)
