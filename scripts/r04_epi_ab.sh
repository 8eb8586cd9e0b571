#!/bin/bash
# The row conv's epilogue: the identity form for the input gradient (no fma when center / scale / shift are
# absent) and 8-byte stores straight from the accumulators (SHPL_ROWS_EPI8, RSTORES = 4), against the round's
# base library: conv parity tests on each, then conv and training bench lines with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=sparse_pooling_amd/variants/libshpl_base.so
E=sparse_pooling_amd/variants/libshpl_epi8.so
N=sparse_pooling_amd/libshpl.so
for v in "id=$N" "epi8=$E"; do
  n=${v%%=*}; lib=${v#*=}
  SHPL_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_epi_tests_$n.log 2>&1 || { tail -30 gpurun_out/r04_epi_tests_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/r04_epi_tests_$n.log)"
done
bash scripts/ab_args.sh r04_econv "--workload conv --dtype bf16" "k_conv_rows|k_pool_runs" "base=$B" "id=$N" "epi8=$E" || exit 1
bash scripts/ab_args.sh r04_etrain "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<|k_bn_" "base=$B" "id=$N" "epi8=$E" "base2=$B" || exit 1
