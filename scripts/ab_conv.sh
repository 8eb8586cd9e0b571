#!/bin/bash
# A/B of the bf16 forward conv: tests, bench lines, PMC passes on the dense kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline > gpurun_out/cb.log 2>&1 || exit 1
grep -o '"unfused.*' gpurun_out/cb.log
B="bench.py --workload conv --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-graph"
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
         "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex 'k_conv3x3<unsigned short, false' -d gpurun_out/ab_pmc_$i -o run \
    --output-format csv -- python3 $B > gpurun_out/ab_pmc_$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_pmc_$i.log; exit $rc; }
done
python3 - <<'PY'
import csv,glob,collections
for f in sorted(glob.glob('gpurun_out/ab_pmc_*/**/*counter_collection.csv',recursive=True)):
    acc=collections.defaultdict(list)
    for r in csv.DictReader(open(f)): acc[r['Counter_Name']].append(float(r['Counter_Value']))
    for k,v in acc.items(): print(f.split('/')[1], k, sum(v)/len(v))
PY
