#!/bin/bash
# BatchNorm apply-kernel A/B: training benches + BN kernel times from one rocprof pass each dtype.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for dt in f32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bn_$dt -o run --output-format csv -- \
    python3 bench.py --workload conv --train --dtype $dt --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bn_$dt.log 2>&1 || exit 1
  grep '^{' gpurun_out/prof_bn_$dt.log | cut -c1-200
  python3 - $dt <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/prof_bn_{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_bn' in r['Name'] or 'k_conv3x3' in r['Name'] or 'wgrad' in r['Name']: print(' ', r['Name'][30:100], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
PY
done
