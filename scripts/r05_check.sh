#!/bin/bash
# Round 5: the whole GPU suite + smoke on the current tree, then the config 2 / 5 / 6 bench lines (regression
# check of the index-kernel changes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05_smoke.log
for c in 2 5 6; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/r05_check_c$c.log 2>&1 || { tail -5 gpurun_out/r05_check_c$c.log; exit 1; }
  grep '^{' gpurun_out/r05_check_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c$c', d['value'], d['ms_per_step'], r['frac'], (d.get('frame_checksums') or {}).get('match_n1'))"
done
echo done
