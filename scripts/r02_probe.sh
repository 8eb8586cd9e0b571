#!/bin/bash
# Round-2 first probe: parity tests, default bench, per-rank frame counts of
# config-4 strong scaling (64/w frames at w = 8, 4, 2), config-3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
for f in 8 16 32; do
  timeout -k 10 300 python bench.py --frames $f --steps 50 --no-cpu-baseline > gpurun_out/bench_f$f.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_f$f.log | cut -c1-300
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit $?
tail -1 gpurun_out/prof_c3.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f8 -o run --output-format csv -- \
  python3 bench.py --frames 8 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_f8.log 2>&1 || exit $?
echo done
