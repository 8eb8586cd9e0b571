#!/bin/bash
# Round 4, first GPU pass on the pruned library: the oracle-pinned checksum tables, the whole GPU suite,
# smoke, and the BASELINE-config bench lines with their CPU baselines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_checksums_oracle.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_checksums_oracle.log 2>&1
rc=$?; echo "checksum tests rc=$rc"; tail -3 gpurun_out/r04_checksums_oracle.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04_checksums_oracle.log | head; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04_gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r04_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04_smoke.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/r04_bench_$n.log 2>&1 || { tail -5 gpurun_out/r04_bench_$n.log; exit 1; }
  grep '^{' gpurun_out/r04_bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$n', d['value'], d['unit'], d['ms_per_step'], r['frac'], r.get('traffic'), (d.get('frame_checksums') or {}).get('match_n1'), c.get('value'), c.get('kind'))"
}
run default
run c3 --config 3 --steps 200
run c5 --config 5
echo done
