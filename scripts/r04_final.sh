#!/bin/bash
# Round 4 evidence on the final tree: the whole GPU suite, smoke, every bench workload, kernel traces of the
# headline, config 3, the bf16 conv and the bf16 training step; the f32 conv's bench line and PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$n.log 2>&1 || { tail -5 gpurun_out/bench_$n.log; exit 1; }
  grep '^{' gpurun_out/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['value'], d['unit'], d['ms_per_step'], r['frac'], r.get('traffic'), (d.get('frame_checksums') or {}).get('match_n1'))"
}
run default
run c3 --config 3 --steps 200
run c5 --config 5
run frames_f64 --workload frames --no-cpu-baseline
run frames_bev --workload frames --maps-form bev_input
run conv_bf16 --workload conv --dtype bf16 --no-cpu-baseline
run train_bf16 --workload conv --train --dtype bf16 --no-cpu-baseline
run c2f8 --frames 8 --no-cpu-baseline
run conv_f32 --workload conv --no-cpu-baseline
trace() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- \
    python3 bench.py "$@" --no-cpu-baseline > gpurun_out/prof_$n.log 2>&1 || { tail -5 gpurun_out/prof_$n.log; exit 1; }
  echo "trace $n ok"
}
trace c2 --steps 20 --warmup 2
trace c3 --config 3 --steps 100
trace conv_bf16 --workload conv --dtype bf16
trace train_bf16 --workload conv --train --dtype bf16 --steps 10
DT=f32 bash scripts/gpu_conv_prof.sh || exit 1
echo done
