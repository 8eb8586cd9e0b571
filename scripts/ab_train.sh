#!/bin/bash
# conv tests, then the training benches (f32, bf16) and one rocprof stats pass of the bf16 one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for dt in f32 bf16; do
  timeout -k 10 300 python bench.py --workload conv --train --dtype $dt --no-cpu-baseline > gpurun_out/tr_$dt.log 2>&1 || { tail -5 gpurun_out/tr_$dt.log; exit 1; }
  grep '^{' gpurun_out/tr_$dt.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$dt', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tr -o run --output-format csv -- \
  python3 bench.py --workload conv --train --dtype bf16 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tr.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/prof_tr/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('reduce','finalize')): print(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, 'us')
PY
