#!/bin/bash
# k_once's gathered-row re-fetch at config 6: FETCH_SIZE of the library (base) and of the XCD-contiguous block
# order (variants/libshpl_oncexcd.so), one pass each; k_once's fetch per launch printed (x2 gfx950 correction).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in base=sparse_pooling_amd/libshpl.so xcd=sparse_pooling_amd/variants/libshpl_oncexcd.so; do
  n=${spec%%=*}; lib=$PWD/${spec#*=}
  SHPL_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_once" \
    -d gpurun_out/pmc_once_$n -o run --output-format csv -- \
    python3 bench.py --config 6 --no-pool-report --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_once_$n.log 2>&1
  rc=$?; echo "pmc once $n rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_once_$n.log; exit $rc; }
  f=$(find gpurun_out/pmc_once_$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if r["Counter_Name"] == "FETCH_SIZE"]
print(sys.argv[2], "k_once launches", len(v), "fetch MB per launch (x2):", [round(2 * x * 1024 / 1e6, 1) for x in v])
PY
done
echo done
