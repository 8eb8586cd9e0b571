#!/bin/bash
# BatchNorm apply streams (bf16): rows in flight per iteration (SHPL_BN_FWD_U / SHPL_BN_BWD_U) and rows per
# thread (SHPL_BN_RPT) against the library's 4 / 2 / 8, on the training step. Measured, none faster
# (profiles/r04_bnu_ab.log); the switches were removed again.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=sparse_pooling_amd/variants
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py -x -q -k "batch_norm or fused_conv_autograd" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_bnu_tests.log 2>&1 || { tail -30 gpurun_out/r04_bnu_tests.log; exit 1; }
for v in u84 u44 r16 u84r16; do
  SHPL_LIB=$V/libshpl_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py -x -q -k "batch_norm or fused_conv_autograd" --timeout 300 --timeout-method thread -p no:cacheprovider >> gpurun_out/r04_bnu_tests.log 2>&1 || { tail -30 gpurun_out/r04_bnu_tests.log; exit 1; }
done
echo "tests: $(grep -c passed gpurun_out/r04_bnu_tests.log) runs passed"
bash scripts/ab_args.sh r04_bnu "--workload conv --train --dtype bf16 --steps 10" "k_bn_apply_vec|k_bn_bwd_apply_vec|k_bn_bwd_partial" \
  "base=$N" "u84=$V/libshpl_u84.so" "u44=$V/libshpl_u44.so" "r16=$V/libshpl_r16.so" "u84r16=$V/libshpl_u84r16.so" "base2=$N" || exit 1
