#!/bin/bash
# Round 3: bucketed pulls (shpl_build_index_buckets + shpl_pull_buckets, one stream) -- parity, then
# config 3 A/B against the range CSR + k_rows path (--no-buckets), and a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "bucket or backward or ragged" > gpurun_out/bkt_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/bkt_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/bkt_tests.log | head -30; exit $rc; }
for v in bkt csr bkt csr; do
  extra=""; [ "$v" = csr ] && extra="--no-buckets"
  timeout -k 10 300 python bench.py --config 3 --steps 200 --no-cpu-baseline $extra > gpurun_out/c3_$v.log 2>&1 || { tail -5 gpurun_out/c3_$v.log; exit 1; }
  tail -1 gpurun_out/c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'), d['frame_checksums']['match_n1'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bkt -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 50 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bkt.log 2>&1 || exit 1
echo done
