#!/bin/bash
# Round 6: config 3's pull pairs as independent 64-entry window waves (k_seg2, SHPL_PAIR_SEG=1 variant) against
# k_rows2: parity of the variant (bucketed pipeline, ragged and short-stretch batches, config-3 checksum
# table), then the bench line and kernel trace of each library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-sparse_pooling_amd/variants/libshpl_seg.so}
N=sparse_pooling_amd/libshpl.so
SHPL_LIB=$V timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "test_pipeline_backward_matches_oracle or test_bucket_pulls_ragged_batch or test_window_pulls" \
  tests/test_gpu_checksums_oracle.py > gpurun_out/r06_seg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_seg_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r06_seg_tests.log | head -20; exit $rc; }
bash scripts/ab_kernels.sh r06_seg "--config 3 --steps 200" "k_index1|k_bsort2|k_rows2|k_seg2" rows2=$N seg=$V rows2b=$N segb=$V
