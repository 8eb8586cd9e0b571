#!/bin/bash
# Round 6: the occupancy-limited input gradient skipping the MFMAs of dead output rows (SHPL_ROWS_DEAD3) against
# computing every row (variants/libshpl_nodead3.so), then the side-stream placements of the bf16 training
# backward again; the conv-gradient tests first. Bench lines interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r06_dead3; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1
rc=$?; tail -1 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $o/tests.log | head; exit $rc; }
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  SHPL_LIB=$lib timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline "$@" > $o/bench_$n.log 2>&1 || { tail -5 $o/bench_$n.log; exit 1; }
  grep '^{' $o/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['ms_per_step'], r['frac'])"
}
L=sparse_pooling_amd/libshpl.so; V=sparse_pooling_amd/variants/libshpl_nodead3.so
for k in 1 2; do
  run dead3_$k $L
  run all_$k $V
  run wside_$k $L --wgrad-side on
  run nozero_$k $L --img-zero-side off
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- \
  python3 bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
f=$(find $o/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "shpl" in r["Name"] and float(r["AverageNs"]) > 50e3:
        print("  ", r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
echo done
