#!/bin/bash
# Training backward: the weight gradient on a side stream beside the input gradient (FusionConv.WGRAD_BESIDE,
# default) against after it on one stream (--wgrad-after): conv gradient parity, then the training step.
# Measured and dropped (profiles/r04_wside_ab.log); the switch was removed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_wside_tests.log 2>&1 || { tail -30 gpurun_out/r04_wside_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_wside_tests.log)"
bash scripts/ab_args.sh r04_wside "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows<2|k_wgrad_rows<|k_pool_runs|k_occ|k_dense" \
  "after=$N|--wgrad-after" "beside=$N" "after2=$N|--wgrad-after" "beside2=$N" || exit 1
