#!/bin/bash
# Training step: the image gradient's zeros from few waves on a high-priority side stream beside the forward
# conv (shpl_zero_fill, FusionConv.DIMG_WAVES) against the whole pull in the backward (--dimg-waves 0).
# Measured and dropped (profiles/r04_dimg_ab.log: three runs, the last with the fill's buffer handed to
# autograd without other references); shpl_zero_fill and the switch were removed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dimg_tests.log 2>&1 || { tail -30 gpurun_out/r04_dimg_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_dimg_tests.log)"
bash scripts/ab_args.sh r04_dimg "--workload conv --train --dtype bf16 --steps 10" "k_zero_stream|k_dense|k_sparse<|k_conv_rows<4, 2" \
  "w0=$N|--dimg-waves 0" "w256=$N|--dimg-waves 256" "w1024=$N|--dimg-waves 1024" "w0b=$N|--dimg-waves 0" "w256b=$N|--dimg-waves 256" || exit 1
