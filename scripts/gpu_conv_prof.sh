#!/bin/bash
# rocprofv3 evidence for the post-fusion conv workload (bench.py --workload conv):
# kernel-trace stats, then one PMC pass per counter group (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass), kernel filter on the conv call's kernels.
# Each pass has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DT="${DT:-f32}"
CFG="${CFG:-2}"  # 6: RetinaNet's 512 -> 256 conv (k_conv_wide for bf16); tags conv_c6_<dt>
T=$DT; [ "$CFG" = 6 ] && T=c6_$DT
B="bench.py --workload conv --config $CFG --dtype $DT --steps 3 --warmup 1 --no-cpu-baseline --no-graph"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_conv_$T -o run --output-format csv -- \
  python3 bench.py --workload conv --config $CFG --dtype $DT --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_conv_$T.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex 'k_conv3x3|k_conv_rows|k_conv_wide|k_pool_runs|k_occ_frame|k_pack_w' -d gpurun_out/pmc_conv_${T}_$i -o run \
    --output-format csv -- python3 $B > gpurun_out/pmc_conv_${T}_$i.log 2>&1
  rc=$?; echo "pmc '$c' rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
