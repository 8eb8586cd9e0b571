#!/bin/bash
# k_csr_frame phase costs: kernel traces of the index-only loop (scripts/csr_probe.py) on the library and on the
# probe variants that return after the histogram + scan (SHPL_CSR_PROBE=1) and after the placement (=2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in full csrp1 csrp2; do
  lib=sparse_pooling_amd/libshpl.so; [ $v = full ] || lib=sparse_pooling_amd/variants/libshpl_$v.so
  SHPL_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/csrp_$v -o run --output-format csv -- \
    python3 scripts/csr_probe.py > gpurun_out/csrp_$v.log 2>&1 || { tail -5 gpurun_out/csrp_$v.log; exit 1; }
  f=$(find gpurun_out/csrp_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_csr_frame" in r["Name"]:
        print(sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["MinNs"]) / 1e3, 2))
PY
done
