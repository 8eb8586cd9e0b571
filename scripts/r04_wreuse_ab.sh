#!/bin/bash
# Training backward (bf16): the weight gradient reading the forward's pooled operand (shpl_conv3x3_wgrad_reuse,
# default) against preparing its own (--no-wgrad-reuse): conv gradient parity, then the training step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_wreuse_tests.log 2>&1 || { tail -30 gpurun_out/r04_wreuse_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_wreuse_tests.log)"
bash scripts/ab_args.sh r04_wreuse "--workload conv --train --dtype bf16 --steps 10" "k_wgrad_rows<|k_pool_runs|k_occ" \
  "own=$N|--no-wgrad-reuse" "reuse=$N" "own2=$N|--no-wgrad-reuse" "reuse2=$N" || exit 1
