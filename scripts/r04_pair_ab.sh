#!/bin/bash
# k_conv_pair (two waves per workgroup, 16x16x32 MFMAs) vs k_conv_rows: conv parity tests, then conv and
# training bench lines with kernel traces for both libraries; then the raw-scan timeline (r04_frames_trace.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_pair_tests.log 2>&1 || { tail -30 gpurun_out/r04_pair_tests.log; exit 1; }
tail -1 gpurun_out/r04_pair_tests.log
R=sparse_pooling_amd/variants/libshpl_rows.so
N=sparse_pooling_amd/libshpl.so
bash scripts/ab_args.sh r04_pconv "--workload conv --dtype bf16" "k_conv_rows|k_conv_pair|k_pool_runs" "rows=$R" "pair=$N" "rows2=$R" "pair2=$N" || exit 1
bash scripts/ab_args.sh r04_ptrain "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_conv_pair|k_wgrad_rows<|k_bn_" "rows=$R" "pair=$N" || exit 1
bash scripts/r04_frames_trace.sh
