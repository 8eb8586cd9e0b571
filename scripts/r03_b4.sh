#!/bin/bash
# Round 3 batch 4: bucket CSR (parallel count reading, 512-thread sorts) vs the range CSR at
# config 3; the raw-scan step's kernel trace (maps after the streaming pass); the EPI8 probes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "ragged or row_keyed or long_run or empty_map or backward or velodyne" > gpurun_out/b4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/b4_tests.log; [ $rc -eq 0 ] || exit $rc
for p in range bucket range bucket; do
  timeout -k 10 300 python bench.py --config 3 --steps 100 --no-cpu-baseline --csr-path $p > gpurun_out/c3_$p.log 2>&1 || { tail -5 gpurun_out/c3_$p.log; exit 1; }
  tail -1 gpurun_out/c3_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$p', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline --no-graph > gpurun_out/prof_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fr -o run --output-format csv -- \
  python3 bench.py --workload frames --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_fr.log 2>&1 || exit 1
for v in epi8; do
  SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k rows > gpurun_out/$v.log 2>&1
  echo "$v rows tests rc=$?"; tail -2 gpurun_out/$v.log
done
echo done
