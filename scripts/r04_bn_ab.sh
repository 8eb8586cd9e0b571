#!/bin/bash
# Training step: BatchNorm vector kernels with their switches at compile time (the library at HEAD: run-time
# flags), and the image gradient's zeros streamed beside the forward conv (--dimg-after: in the backward's pull;
# that switch and its side-stream pass were removed after this run: step 7.44 -> 8.03 ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
H=sparse_pooling_amd/variants/libshpl_head.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_bn_tests.log 2>&1 || { tail -30 gpurun_out/r04_bn_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_bn_tests.log)"
bash scripts/ab_args.sh r04_bn "--workload conv --train --dtype bf16 --steps 10" "k_bn|k_dense|k_sparse<|k_conv_rows|k_wgrad_rows<" \
  "head=$H|--dimg-after" "bn=$N|--dimg-after" "zero=$H" "both=$N" "head2=$H|--dimg-after" "both2=$N" || exit 1
