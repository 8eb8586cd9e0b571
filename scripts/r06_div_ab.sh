#!/bin/bash
# Round 6: two index-chain trims at config 3 -- the stride divisions as exact multiplies for power-of-two strides,
# and the bucket words carrying their entries' source rows and values (the bucket sort then reads them in the
# words' round trip instead of gathering them): parity on the shipped library (both), then bench + trace of
# r5idx (neither), nopow (bucket sources only, SHPL_POW2_DIV=0) and the shipped library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
A=sparse_pooling_amd/variants/libshpl_r5idx.so
B=sparse_pooling_amd/variants/libshpl_nopow.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "index or golden or test_pipeline_backward_matches_oracle or ragged or kitti or mv3d or window or barrier" \
  tests/test_gpu_checksums_oracle.py > gpurun_out/r06_div_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_div_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06_div_tests.log | head; exit $rc; }
bash scripts/ab_kernels.sh r06_div5 "--config 3 --steps 200" "k_index1|k_bsort2" r5idx=$A now=$N r5idxb=$A nowb=$N
