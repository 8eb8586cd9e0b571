#!/bin/bash
# A/B of k_conv_rows variants (sparse_pooling_amd/variants/<v>.so) on the bf16 conv workload:
# fused conv ms (shpl_conv3x3 call: prep + kernel) and the dense conv over bv_fused.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-1}); do
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps ${STEPS:-10} ${BENCH_ARGS} > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', r.get('kernel_ms'), d['unfused']['conv_ms'], d['unfused'].get('bitwise_equal'))"
done
done
