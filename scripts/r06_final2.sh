#!/bin/bash
# Round 6 evidence on the final tree, part 2: rocprofv3 kernel traces (--kernel-trace --stats) of the headline,
# config 3, config 6, the bf16 convs and the bf16 training step; then the PMC passes (FETCH_SIZE and
# WRITE_SIZE in runs of their own) of every workload the bench looks up in profiles/traffic.json, and the conv
# calls' (scripts/gpu_conv_prof.sh: bf16, f32, the RetinaNet bf16 conv).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
trace() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_$n -o run --output-format csv -- \
    python3 bench.py "$@" --no-cpu-baseline > gpurun_out/r06_prof_$n.log 2>&1 || { tail -5 gpurun_out/r06_prof_$n.log; exit 1; }
  echo "trace $n ok"
}
trace c2 --steps 20 --warmup 2
trace c3 --config 3 --steps 100
trace c6 --config 6 --steps 10
trace conv_bf16 --workload conv --dtype bf16
trace conv_c6_bf16 --workload conv --config 6 --dtype bf16 --steps 5
trace train_bf16 --workload conv --train --dtype bf16 --steps 10
WHICH="c2f64 c2f8 c3f4 c5f64 frf64 frbev trbf16" bash scripts/r03_pmc.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "shpl" -d gpurun_out/pmc_c6f64_$c -o run --output-format csv -- \
    python3 bench.py --config 6 --no-pool-report --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_c6f64_$c.log 2>&1
  rc=$?; echo "pmc c6f64 $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_c6f64_$c.log; exit $rc; }
done
DT=bf16 bash scripts/gpu_conv_prof.sh || exit 1
DT=f32 bash scripts/gpu_conv_prof.sh || exit 1
CFG=6 DT=bf16 bash scripts/gpu_conv_prof.sh || exit 1
echo done
