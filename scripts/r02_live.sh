# The sparse passes over each frame's live entries (SHPL_LIVE=1, default) vs the whole capacity (0):
# GPU tests, then frames / config-2 / config-5 A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/live; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/live/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/live/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  export SHPL_LIVE=$v
  for w in "--workload frames" "--config 2" "--config 5"; do
    tag=$(echo "$w" | tr -d ' -')
    timeout -k 10 300 python bench.py $w --no-cpu-baseline --steps 20 > gpurun_out/live/${tag}_$v.log 2>&1 || { tail -3 gpurun_out/live/${tag}_$v.log; exit 1; }
    grep '^{' gpurun_out/live/${tag}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('live=$v $tag', d['ms_per_step'], d['roofline']['frac'], d.get('stages_ms',{}).get('k_sparse_ms'), (d.get('frame_checksums') or {}).get('match_n1'))"
  done
done
