#!/bin/bash
# Config-3 iteration: GPU tests, config-3 bench, its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTSEL:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 3 --steps 50 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c3.log | cut -c1-600
timeout -k 10 300 python bench.py --config 3 --steps 50 --no-cpu-baseline --no-graph > gpurun_out/bench_c3_eager.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c3_eager.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager', d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit 1
echo done
