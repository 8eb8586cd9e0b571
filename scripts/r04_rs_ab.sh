#!/bin/bash
# (The switch was removed from the sources after this measurement.)
# Register-staged rows (SHPL_ROWS_RS: dense sources of <= 2 chunks -- the input gradient -- load their rows into
# VGPRs and ds_write them, no LDS-DMA in the loop) against the LDS-DMA ring: conv parity on the new library,
# then training and conv bench lines with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
D=sparse_pooling_amd/variants/libshpl_dma.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_rs_tests.log 2>&1 || { tail -30 gpurun_out/r04_rs_tests.log; exit 1; }
echo "rs: $(tail -1 gpurun_out/r04_rs_tests.log)"
bash scripts/ab_args.sh r04_rstrain "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<" "dma=$D" "rs=$N" "dma2=$D" "rs2=$N" || exit 1
