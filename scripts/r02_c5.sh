cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "batch_matches or config5 or backward" > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for a in "" "--no-interleave" "" "--no-interleave"; do
timeout -k 10 300 python bench.py --config 5 --steps 10 --no-cpu-baseline $a > gpurun_out/c5.log 2>&1 || exit 1
tail -1 gpurun_out/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[$a]', d['ms_per_step'], r['frac'], r.get('k_dense_ms'), r.get('k_sparse_ms'))"
done
