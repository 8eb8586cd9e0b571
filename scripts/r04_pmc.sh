#!/bin/bash
# Round-4 PMC refresh on the final library: every bench workload (scripts/r03_pmc.sh, CONV=bf16), then
# config 6 (the RetinaNet P2 shape) and its bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CONV=bf16 bash scripts/r03_pmc.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "shpl" -d gpurun_out/pmc_c6f64_$c -o run --output-format csv -- \
    python3 bench.py --config 6 --no-pool-report --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_c6f64_$c.log 2>&1
  rc=$?; echo "pmc c6f64 $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_c6f64_$c.log; exit $rc; }
done
timeout -k 10 400 python bench.py --config 6 > gpurun_out/bench_c6.log 2>&1 || { tail -5 gpurun_out/bench_c6.log; exit 1; }
echo done
