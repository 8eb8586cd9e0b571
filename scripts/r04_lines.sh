#!/bin/bash
# Bench lines after the PMC stamps (traffic on every line): the bf16 training step (its corrected byte count),
# the f32 conv and config 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > gpurun_out/bench_train_bf16.log 2>&1 || { tail -5 gpurun_out/bench_train_bf16.log; exit 1; }
timeout -k 10 400 python bench.py --workload conv --no-cpu-baseline > gpurun_out/bench_conv_f32.log 2>&1 || { tail -5 gpurun_out/bench_conv_f32.log; exit 1; }
timeout -k 10 400 python bench.py --config 6 > gpurun_out/bench_c6.log 2>&1 || { tail -5 gpurun_out/bench_c6.log; exit 1; }
for n in train_bf16 conv_f32 c6; do
  grep '^{' gpurun_out/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), r.get('algorithmic_bytes_per_step'))"
done
