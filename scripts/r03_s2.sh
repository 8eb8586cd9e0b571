#!/bin/bash
# Round 3, session 2, first GPU pass on the restored HEAD: the whole GPU suite, smoke,
# the default bench (both CPU-baseline legs), config 3 and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/bench.log | cut -c1-600
timeout -k 10 300 python bench.py --config 3 --steps 100 --no-cpu-baseline > gpurun_out/c3.log 2>&1 || exit 1
grep '^{' gpurun_out/c3.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit 1
echo done
