#!/bin/bash
# PMC of the raw-scan step's k_dense beside the index chain (default) and alone
# (--dense-after csr: the chain first), one counter group per run: HBM bytes, L2 hit / miss, wave and
# wait cycles, clock. Plus the counter list of this box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_dpmc
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r04_dpmc/counters.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  for v in "beside|" "after|--dense-after csr"; do
    n=${v%%|*}; a=${v#*|}
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_dense" -d gpurun_out/r04_dpmc/${n}_$i -o run --output-format csv -- \
      python3 bench.py --workload frames --maps-form bev_input --steps 5 --warmup 1 --no-cpu-baseline $a > gpurun_out/r04_dpmc/${n}_$i.log 2>&1
    rc=$?; echo "pmc $n '$grp' rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r04_dpmc/${n}_$i.log; exit $rc; }
  done
done
echo done
