#!/bin/bash
# Round 6: RetinaNet's bf16 conv (k_conv_wide) -- static s_setprio 1 for waves 4-7 (SHPL_WIDE_PRIO=1 variant)
# against the shipped kernel: the two conv tests on the variant, then bench line + kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-sparse_pooling_amd/variants/libshpl_prio.so}
N=sparse_pooling_amd/libshpl.so
SHPL_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_conv.py -k "retinanet or wide" > gpurun_out/r06_wide_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_wide_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_kernels.sh r06_wide "--workload conv --config 6 --dtype bf16 --steps 10" "k_conv_wide" base=$N prio=$V baseb=$N priob=$V
