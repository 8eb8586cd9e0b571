#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash, abort or timeout ends the
# script (no further GPU work), plain test failures do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; ok $rc || exit $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/prof.log; ok $rc || exit $rc ;;
    pmc)
      # HBM traffic of the SHPL kernels: FETCH_SIZE and WRITE_SIZE in separate passes
      # (they do not fit one TCC pass), kernel filter on the shpl kernels only.
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex 'k_dense|k_sparse|k_csr_frame|k_compact|k_count' \
          -d gpurun_out/pmc_$c -o run --output-format csv -- \
          python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_$c.log 2>&1
        rc=$?; echo "pmc $c rc=$rc"; tail -1 gpurun_out/pmc_$c.log | cut -c1-200; ok $rc || exit $rc
      done ;;
  esac
done
