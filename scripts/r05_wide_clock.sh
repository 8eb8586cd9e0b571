#!/bin/bash
# Round 5: calibration of the wide conv -- hipBLASLt GEMM of the same shape, and the effective clock of
# k_conv_wide (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES) from a PMC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_calib.py 2>&1 | tee gpurun_out/r05_gemm_calib.log
for v in base wide8; do
  lib=""; [ $v != base ] && lib=sparse_pooling_amd/variants/lib_$v.so
  SHPL_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU --kernel-include-regex "conv_wide" -d gpurun_out/r05_wide_clk_$v -o run --output-format csv -- \
    python3 bench.py --workload conv --config 6 --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/r05_wide_clk_$v.log 2>&1
  echo "pmc $v rc=$?"
done
echo done
