#!/bin/bash
# Band sums of the statistics forms in registers across the band (SHPL_ROWS_STREG=2) against per-lane LDS sums
# (SHPL_ROWS_STREG=1, the library): conv parity on the variant, then the training step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=sparse_pooling_amd/variants/libshpl_streg2.so
N=sparse_pooling_amd/libshpl.so
SHPL_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_streg2_tests.log 2>&1 || { tail -30 gpurun_out/r04_streg2_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_streg2_tests.log)"
bash scripts/ab_args.sh r04_streg2 "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows<4, 2, true, false, true" "lds=$N" "reg=$V" "lds2=$N" "reg2=$V" || exit 1
