#!/bin/bash
# Round-2 evidence. PART=tests: the GPU test suite and smoke(); PART=bench: the bench
# lines of every workload, each beside a rocprofv3 --kernel-trace --stats run of the
# same command. Everything lands in gpurun_out/ev/ (copied into profiles/r02_* after).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
O=gpurun_out/ev
if [ "${PART:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  exit 0
fi
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | cut -c1-240
  if [ -n "$PROF" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- \
      python3 bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_$n.log 2>&1 || { tail -5 $O/prof_$n.log; exit 1; }
    echo "prof $n ok"
  fi
}
for w in ${WORKLOADS:-default config3 config5 frames conv conv_bf16 train train_bf16}; do
  case $w in
    default) run default ;;
    config3) run config3 --config 3 ;;
    config5) run config5 --config 5 ;;
    frames) run frames --workload frames ;;
    conv) run conv --workload conv ;;
    conv_bf16) run conv_bf16 --workload conv --dtype bf16 ;;
    train) run train --workload conv --train ;;
    train_bf16) run train_bf16 --workload conv --train --dtype bf16 ;;
  esac
done
echo done
