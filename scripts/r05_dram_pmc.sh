#!/bin/bash
# Round 5: which part of FETCH_SIZE reaches DRAM. FETCH_SIZE counts every L2 -> fabric read request, Infinity
# Cache (MALL) hits included; TCC_EA0_RDREQ_DRAM counts the requests destined for DRAM. One PMC pass per
# workload (4 TCC counters: RDREQ, RDREQ_DRAM, BUBBLE = 128-byte requests, RDREQ_32B), kernel-filtered.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum"
pass() {  # tag, regex, bench args...
  local t=$1 re=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$re" -d gpurun_out/pmcd_$t -o run --output-format csv -- \
    python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmcd_$t.log 2>&1
  rc=$?; echo "pmc $t rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmcd_$t.log; exit $rc; }
}
pass c2 "k_dense|k_sparse" --config 2 --no-pool-report
pass conv_bf16 "k_conv_rows|k_pool_runs" --workload conv --dtype bf16
pass conv_c6_bf16 "k_conv_wide|k_pool_runs_wide" --workload conv --config 6 --dtype bf16
pass train_bf16 "shpl" --workload conv --train --dtype bf16
pass c3 "k_rows2|k_index1|k_bsort2" --config 3
pass c6 "k_dense|k_once" --config 6 --no-pool-report
echo done
