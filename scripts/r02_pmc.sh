#!/bin/bash
# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each) of the SHPL kernels for
# one bench workload: gpurun_out/pmc_<tag>_<counter>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-c5}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-k_dense|k_sparse|k_rows|k_csr|k_compact|k_count|k_zero}" \
    -d gpurun_out/pmc_${TAG}_$c -o run --output-format csv -- \
    python3 bench.py ${BENCH_ARGS:---config 5} --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?; echo "pmc $TAG $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_${TAG}_$c.log; exit $rc; }
done
