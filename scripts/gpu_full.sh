#!/bin/bash
# Round-end measurement on the GPU box: parity tests, smoke, the default bench
# line + rocprof kernel stats + PMC traffic, and the other workloads' lines
# (configs 3 / 5, raw scans) with their kernel stats. Each GPU step has its own
# time limit; a crash, abort or timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="tests smoke bench prof pmc" ./scripts/gpu_round.sh || exit $?
run() {  # name, seconds, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -n 1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run bench_c3 300 python bench.py --config 3
run bench_c5 400 python bench.py --config 5
run bench_frames 400 python bench.py --workload frames
run bench_noov 300 python bench.py --no-overlap --no-graph --no-cpu-baseline
run bench_conv 400 python bench.py --workload conv
run bench_conv_bf16 300 python bench.py --workload conv --dtype bf16 --no-cpu-baseline
run bench_conv_train 300 python bench.py --workload conv --train
for c in 3 5; do
  run prof_c$c 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o run --output-format csv -- \
    python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline
done
run prof_frames 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frames -o run --output-format csv -- \
  python3 bench.py --workload frames --steps 10 --warmup 2 --no-cpu-baseline
echo all done
