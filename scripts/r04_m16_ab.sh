#!/bin/bash
# The row conv with v_mfma_f32_16x16x32_bf16 (SHPL_ROWS_M16, even chunk counts without statistics) against
# 32x32x16 (same tree, SHPL_ROWS_M16=0) and the committed library: conv parity on the new one, then conv and
# training bench lines with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
H=sparse_pooling_amd/variants/libshpl_head.so
M=sparse_pooling_amd/variants/libshpl_m32.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_m16_tests.log 2>&1 || { tail -30 gpurun_out/r04_m16_tests.log; exit 1; }
echo "m16: $(tail -1 gpurun_out/r04_m16_tests.log)"
bash scripts/ab_args.sh r04_m16conv "--workload conv --dtype bf16" "k_conv_rows" "head=$H" "m32=$M" "m16=$N" "head2=$H" "m16b=$N" || exit 1
bash scripts/ab_args.sh r04_m16train "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<" "head=$H" "m16=$N" "head2=$H" "m16b=$N" || exit 1
