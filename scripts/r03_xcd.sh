#!/bin/bash
# Round 3: XCD-contiguous row blocks in k_rows (config 3) -- parity subset, then A/B against the
# blockIdx-order variant (SHPL_PULL_XCD=0), and a PMC pass of the config-3 step for the fetch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "ragged or row_keyed or long_run or empty_map or backward" > gpurun_out/xcd_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/xcd_tests.log; [ $rc -eq 0 ] || exit $rc
for v in default noxcd default noxcd; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 300 python bench.py --config 3 --steps 200 --no-cpu-baseline > gpurun_out/c3_$v.log 2>&1 || { tail -5 gpurun_out/c3_$v.log; exit 1; }
  tail -1 gpurun_out/c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'), d['frame_checksums']['match_n1'])"
done
unset SHPL_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3x -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3x.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/pmc_c3x -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_c3x.log 2>&1 || exit 1
echo done
