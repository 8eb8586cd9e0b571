#!/bin/bash
# The row-conv kernels without the per-step vmcnt ladder: conv / training parity, then conv and training
# bench lines for the previous form (SHPL_ROWS_WLATE=1) and the new one, with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_conv_tests.log 2>&1 || { tail -30 gpurun_out/r04_conv_tests.log; exit 1; }
tail -1 gpurun_out/r04_conv_tests.log
W=sparse_pooling_amd/variants/libshpl_wlate.so
N=sparse_pooling_amd/libshpl.so
bash scripts/ab_args.sh r04_conv "--workload conv --dtype bf16" "k_conv_rows|k_pool_runs" "wlate=$W" "new=$N" "wlate2=$W" "new2=$N" || exit 1
bash scripts/ab_args.sh r04_train "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<|k_bn_" "wlate=$W" "new=$N" || exit 1
