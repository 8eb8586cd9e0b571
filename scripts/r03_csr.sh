#!/bin/bash
# Round 3 batch 3: the bucket CSR (parity subset, then config 3 with each builder),
# and the 8-byte-store epilogue probes (as rebuilt; + RSTORES=4; + drained ring waits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/csr_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/csr_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/csr_tests.log | head -20; exit $rc; }
for p in auto range bucket auto range bucket; do
  timeout -k 10 300 python bench.py --config 3 --steps 100 --no-cpu-baseline --csr-path $p > gpurun_out/c3_$p.log 2>&1 || { tail -5 gpurun_out/c3_$p.log; exit 1; }
  tail -1 gpurun_out/c3_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$p', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'), d['frame_checksums']['match_n1'])"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline > gpurun_out/frames_$r.log 2>&1 || { tail -5 gpurun_out/frames_$r.log; exit 1; }
  tail -1 gpurun_out/frames_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('frames', d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_frac'], d['stages_ms'], d['frame_checksums']['match_n1'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit 1
for v in epi8 epi8r4 epi8drain; do
  SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k rows > gpurun_out/$v.log 2>&1
  echo "$v rows tests rc=$?"; tail -2 gpurun_out/$v.log
done
echo done
