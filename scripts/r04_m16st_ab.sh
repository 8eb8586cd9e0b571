#!/bin/bash
# The statistics forms of the row conv on 16x16x32 MFMAs too (SHPL_ROWS_M16_ST) against the committed library
# (32x32x16 for them): conv parity, then training bench lines with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
H=sparse_pooling_amd/variants/libshpl_head.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_m16st_tests.log 2>&1 || { tail -30 gpurun_out/r04_m16st_tests.log; exit 1; }
echo "m16st: $(tail -1 gpurun_out/r04_m16st_tests.log)"
bash scripts/ab_args.sh r04_m16st "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<" "head=$H" "st=$N" "head2=$H" "st2=$N" || exit 1
