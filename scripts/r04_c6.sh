#!/bin/bash
# Config 6 (the RetinaNet P2 SHPL shape): the bench line writing its per-frame checksum table (copied to
# gpurun_out/ -- the box's profiles/ does not come back), the table pinned to the oracle, a kernel trace and
# the PMC traffic passes (FETCH_SIZE, WRITE_SIZE: one run each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config 6 --write-checksums > gpurun_out/bench_c6.log 2>&1 || { tail -5 gpurun_out/bench_c6.log; exit 1; }
grep '^{' gpurun_out/bench_c6.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c6', d['value'], d['ms_per_step'], r['frac'], (d.get('cpu_baseline') or {}).get('value'))"
cp profiles/frame_checksums.json gpurun_out/frame_checksums_c6.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_checksums_oracle.py -x -v -k "config6" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c6_oracle.log 2>&1 || { tail -20 gpurun_out/c6_oracle.log; exit 1; }
tail -1 gpurun_out/c6_oracle.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c6 -o run --output-format csv -- \
  python3 bench.py --config 6 --no-cpu-baseline > gpurun_out/prof_c6.log 2>&1 || { tail -5 gpurun_out/prof_c6.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "shpl" -d gpurun_out/pmc_c6f64_$c -o run --output-format csv -- \
    python3 bench.py --config 6 --no-pool-report --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_c6f64_$c.log 2>&1
  rc=$?; echo "pmc c6f64 $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_c6f64_$c.log; exit $rc; }
done
echo done
