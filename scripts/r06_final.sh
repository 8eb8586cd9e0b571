#!/bin/bash
# Round 6 evidence on the final tree, part 1: the RetinaNet conv checksum tables (a GPU run: no oracle
# checksum exists for the conv; tolerance-checked against the oracle by tests/test_gpu_conv.py), the whole GPU
# suite, smoke, and every bench line with its cpu_baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TABLES" ]; then  # SKIP_TABLES=1: the committed tables stand (the conv kernels unchanged)
  for dt in bf16 f32; do
    timeout -k 10 300 python bench.py --workload conv --config 6 --dtype $dt --steps 2 --warmup 1 --no-cpu-baseline \
      --write-checksums > gpurun_out/r06_conv_c6_table_$dt.log 2>&1 || { tail -5 gpurun_out/r06_conv_c6_table_$dt.log; exit 1; }
  done
  cp profiles/frame_checksums.json gpurun_out/frame_checksums.json
fi
if [ -z "$BENCH_ONLY" ]; then  # BENCH_ONLY=1: the bench lines alone (e.g. again once traffic.json is re-stamped)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r06_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06_gpu_tests.log | head; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r06_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/r06_smoke.log
fi
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/r06_bench_$n.log 2>&1 || { tail -5 gpurun_out/r06_bench_$n.log; exit 1; }
  grep '^{' gpurun_out/r06_bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$n', d['value'], d['unit'], d['ms_per_step'], r['frac'], r.get('traffic'), (d.get('frame_checksums') or {}).get('match_n1'), c.get('value'), c.get('kind'))"
}
run default
run c3 --config 3 --steps 200
run c5 --config 5
run c6 --config 6
run frames_f64 --workload frames
run frames_bev --workload frames --maps-form bev_input --no-cpu-baseline
run c2f8 --frames 8 --no-cpu-baseline
run conv_bf16 --workload conv --dtype bf16
run conv_f32 --workload conv
run conv_c6_bf16 --workload conv --config 6 --dtype bf16
run conv_c6_f32 --workload conv --config 6 --no-cpu-baseline
run train_bf16 --workload conv --train --dtype bf16
run train_f32 --workload conv --train --no-cpu-baseline
echo done
