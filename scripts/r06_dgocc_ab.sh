#!/bin/bash
# Round 6: the input gradient's pooled channels stored at the occupied cells only (FusionConv.DGRAD_OCC,
# shpl_conv3x3_dgrad_reuse). The conv-gradient tests, then the bf16 training step with and without it,
# interleaved, and one kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06_dgocc
export TMPDIR=/tmp
o=gpurun_out/r06_dgocc
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1
rc=$?; tail -1 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $o/tests.log | head; exit $rc; }
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline "$@" > $o/bench_$n.log 2>&1 || { tail -5 $o/bench_$n.log; exit 1; }
  grep '^{' $o/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['ms_per_step'], r['frac'], r['algorithmic_bytes_per_step'])"
}
run occ
run whole --no-dgrad-occ
run occ2
run whole2 --no-dgrad-occ
for n in occ whole; do
  a=""; [ $n = whole ] && a="--no-dgrad-occ"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_$n -o run --output-format csv -- \
    python3 bench.py --workload conv --train --dtype bf16 --no-cpu-baseline $a > $o/prof_$n.log 2>&1 || { tail -5 $o/prof_$n.log; exit 1; }
  f=$(find $o/prof_$n -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "shpl" in r["Name"] and float(r["AverageNs"]) > 50e3:
        print("  ", sys.argv[2], r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
echo done
