#!/bin/bash
# Config 3 A/B of k_rows2's XCD schedules (SHPL_ROWS2_SCHED: 0 round robin, 1 (side, frame) units per XCD,
# 2 frames per XCD group): bitwise parity of the bucketed step under each library, then the bench step
# (alternating, twice each) and one rocprof kernel trace each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_sched
export TMPDIR=/tmp
V=sparse_pooling_amd/variants
declare -A LIBS=([s0]=sparse_pooling_amd/libshpl.so [s1]=$V/libshpl_sched1.so [s2]=$V/libshpl_sched2.so)
for n in s0 s1 s2; do
  SHPL_LIB=${LIBS[$n]} timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "backward_matches_oracle or bucket_pulls or row_keyed" > gpurun_out/r04_sched/tests_$n.log 2>&1 || { echo "tests $n failed"; tail -20 gpurun_out/r04_sched/tests_$n.log; exit 1; }
  tail -1 gpurun_out/r04_sched/tests_$n.log
done
for rep in 1 2; do
  for n in s0 s1 s2; do
    SHPL_LIB=${LIBS[$n]} timeout -k 10 300 python bench.py --config 3 --steps 400 --no-cpu-baseline > gpurun_out/r04_sched/c3_${n}_$rep.log 2>&1 || { tail -5 gpurun_out/r04_sched/c3_${n}_$rep.log; exit 1; }
    grep '^{' gpurun_out/r04_sched/c3_${n}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', $rep, d['ms_per_step'], r['kernel_ms'], r['frac'], d['frame_checksums']['match_n1'])"
  done
done
for n in s0 s1 s2; do
  SHPL_LIB=${LIBS[$n]} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_sched/prof_$n -o run --output-format csv -- \
    python3 bench.py --config 3 --steps 200 --no-cpu-baseline > gpurun_out/r04_sched/prof_$n.log 2>&1 || { tail -5 gpurun_out/r04_sched/prof_$n.log; exit 1; }
  f=$(find gpurun_out/r04_sched/prof_$n -name "*kernel_stats.csv" | head -1)
  python3 - "$f" $n <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if any(k in r["Name"] for k in ("k_rows2", "k_bsort2", "k_count", "k_compact")):
        print(sys.argv[2], r["Name"][:60], r["Calls"], r["AverageNs"])
PY
done
echo done
