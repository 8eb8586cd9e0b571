#!/bin/bash
# Round 6: k_index1 with each frame's chunk workgroups on one XCD (SHPL_IDX1_XCD=1 variant: the frame barrier's
# atomics and the aggregate loads stay within one L2) against the shipped mapping: parity, then bench + trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-sparse_pooling_amd/variants/libshpl_ixcd.so}
N=sparse_pooling_amd/libshpl.so
SHPL_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "test_pipeline_backward_matches_oracle or test_bucket_pulls_ragged_batch or test_window_pulls or dirty" \
  tests/test_gpu_checksums_oracle.py > gpurun_out/r06_ixcd_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_ixcd_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06_ixcd_tests.log | head; exit $rc; }
bash scripts/ab_kernels.sh r06_ixcd "--config 3 --steps 200" "k_index1|k_bsort2|k_rows2" base=$N ixcd=$V baseb=$N ixcdb=$V
