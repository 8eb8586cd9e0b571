#!/bin/bash
# A/B of compile-time variants on one workload: the parity subset, then REPS bench runs of
# each variant (SHPL_LIB=sparse_pooling_amd/variants/<v>.so; "default" = libshpl.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTSEL:-backward or row_keyed}" > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-default}; do
  for r in $(seq ${REPS:-2}); do
    if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
    timeout -k 10 300 python bench.py ${BENCH_ARGS:---config 3} --steps ${STEPS:-100} --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['frac'], r.get('k_dense_ms'), r.get('k_sparse_ms'), r.get('backward_ms'))"
  done
done
unset SHPL_LIB
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o run --output-format csv -- \
    python3 bench.py ${BENCH_ARGS:---config 3} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ab.log 2>&1 || exit 1
fi
echo done
