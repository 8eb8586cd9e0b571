#!/bin/bash
# PMC passes over k_conv_rows (bf16 conv workload, fused = <4,true,...>, unfused = <4,false,...>):
# one rocprofv3 --pmc run per counter group, each under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --workload conv --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --no-graph"
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'k_conv_rows' -d gpurun_out/pmc_rows_$i -o run \
    --output-format csv -- python3 $B > gpurun_out/pmc_rows_$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
