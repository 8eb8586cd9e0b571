#!/bin/bash
# Round 6, after the image gradient moved beside the weight gradient (Python only, the library unchanged): the
# conv-gradient GPU tests, then the bf16 and f32 training bench lines (with cpu_baseline) for profiles/r06_final.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_gpu_conv.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06_train_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_train_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06_train_tests.log | head; exit $rc; }
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/r06_bench_$n.log 2>&1 || { tail -5 gpurun_out/r06_bench_$n.log; exit 1; }
  grep '^{' gpurun_out/r06_bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$n', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), c.get('value'))"
}
run train_bf16 --workload conv --train --dtype bf16
run train_f32 --workload conv --train --no-cpu-baseline
echo done
