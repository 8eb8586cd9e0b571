#!/bin/bash
# Round 6: the RetinaNet conv's pooled-runs prep with 4 entries per thread (k_pool_runs_wide_k, shipped) against a
# thread per entry (SHPL_WIDE_RUNS_K=1): the wide-conv tests, then the conv_c6 bf16 bench line (its checksums
# against the stored table: bitwise) and a kernel trace of each, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r06_runsk; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "wide or retina or c6" > $o/tests.log 2>&1
rc=$?; tail -1 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $o/tests.log | head; exit $rc; }
V=sparse_pooling_amd/variants
bash scripts/ab_kernels.sh ${TAG:-r06_runsk} "--workload conv --config 6 --dtype bf16" "pool_runs|k_conv_wide" \
  k4=sparse_pooling_amd/libshpl.so k1=$V/libshpl_runs1.so k8=$V/libshpl_runs8.so k16=$V/libshpl_runs16.so \
  k4b=sparse_pooling_amd/libshpl.so k8b=$V/libshpl_runs8.so
