#!/bin/bash
# A/B of library variants on one bench workload: for each NAME=LIB, the bench line (ms/step, roofline frac)
# and a rocprofv3 kernel trace whose per-kernel averages are printed (kernels matching PATTERN).
#   bash scripts/ab_kernels.sh TAG "BENCH ARGS" PATTERN NAME=LIB ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; bargs=$2; pat=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for nl in "$@"; do
  n=${nl%%=*}; lib=${nl#*=}
  SHPL_LIB=$lib timeout -k 10 300 python bench.py $bargs --no-cpu-baseline > $out/bench_$n.log 2>&1 || { tail -5 $out/bench_$n.log; exit 1; }
  grep '^{' $out/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['ms_per_step'], r['frac'], (d.get('frame_checksums') or {}).get('match_n1'))"
  SHPL_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$n -o run --output-format csv -- \
    python3 bench.py $bargs --no-cpu-baseline > $out/prof_$n.log 2>&1 || { tail -5 $out/prof_$n.log; exit 1; }
  f=$(find $out/prof_$n -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$n" "$pat" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        print("  ", sys.argv[2], r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
echo done
