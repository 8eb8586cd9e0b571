#!/bin/bash
# k_csr_frame with each entry's value and source placed beside its word (SHPL_CSR_SV, default) against
# gathering both at emission (SHPL_CSR_SV=0): CSR parity, the index-only loop, the conv and config-2 steps.
# Measured slower and reverted (profiles/r04_sv_ab.log).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=sparse_pooling_amd/variants/libshpl_sv0.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checksums_oracle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_sv_tests.log 2>&1 || { tail -30 gpurun_out/r04_sv_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_sv_tests.log)"
for v in sv0 sv; do
  lib=$N; [ $v = sv0 ] && lib=$O
  SHPL_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/svp_$v -o run --output-format csv -- \
    python3 scripts/csr_probe.py > gpurun_out/svp_$v.log 2>&1 || { tail -5 gpurun_out/svp_$v.log; exit 1; }
  f=$(find gpurun_out/svp_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_csr_frame" in r["Name"]:
        print("probe", sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
bash scripts/ab_args.sh r04_sv_conv "--workload conv --dtype bf16" "k_csr_frame" "sv0=$O" "sv=$N" "sv0b=$O" "svb=$N" || exit 1
bash scripts/ab_args.sh r04_sv_c2 "--steps 20" "k_csr_frame|k_dense" "sv0=$O" "sv=$N" || exit 1
