#!/bin/bash
# The 16x16 statistics forms summing each row straight from the accumulators (SHPL_ROWS_STREG, default) against
# the f32 transpose through the ring slot (SHPL_ROWS_STREG=0): conv parity, then the training step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=sparse_pooling_amd/variants/libshpl_streg0.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_streg_tests.log 2>&1 || { tail -30 gpurun_out/r04_streg_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_streg_tests.log)"
bash scripts/ab_args.sh r04_streg "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows<4, 2, true, false, true" "xpose=$O" "streg=$N" "xpose2=$O" "streg2=$N" || exit 1
