#!/bin/bash
# (The switch was removed from the sources after this measurement; a rebuild of the variant equals the default.)
# The row kernels' quad layout (SHPL_ROWS_QUAD: each DMA quad of lanes reads one 64-byte segment) against the
# piece-major layout: conv parity tests on both, then conv and training bench lines with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=sparse_pooling_amd/variants/libshpl_noquad.so
N=sparse_pooling_amd/libshpl.so
for v in "quad=$N" "noquad=$B"; do
  n=${v%%=*}; lib=${v#*=}
  SHPL_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_quad_tests_$n.log 2>&1 || { tail -30 gpurun_out/r04_quad_tests_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/r04_quad_tests_$n.log)"
done
bash scripts/ab_args.sh r04_qconv "--workload conv --dtype bf16" "k_conv_rows|k_pool_runs" "noquad=$B" "quad=$N" "noquad2=$B" "quad2=$N" || exit 1
bash scripts/ab_args.sh r04_qtrain "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<|k_bn_" "noquad=$B" "quad=$N" || exit 1
