#!/bin/bash
# Round 3: config 3 with 1 / 2 / 4 steps per captured graph (one queue since the bucketed step), after the
# bucket-pull parity subset; then config 2 at 1 and 2 steps per graph.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "bucket_pulls or backward" > gpurun_out/gs_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gs_tests.log; [ $rc -eq 0 ] || exit $rc
for g in 1 2 4 1 2 4; do
  timeout -k 10 300 python bench.py --config 3 --steps 200 --no-cpu-baseline --graph-steps $g > gpurun_out/gs_c3_$g.log 2>&1 || { tail -5 gpurun_out/gs_c3_$g.log; exit 1; }
  tail -1 gpurun_out/gs_c3_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c3 g$g', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'), d['frame_checksums']['match_n1'])"
done
for g in 1 2; do
  timeout -k 10 300 python bench.py --config 2 --steps 20 --no-cpu-baseline --graph-steps $g > gpurun_out/gs_c2_$g.log 2>&1 || { tail -5 gpurun_out/gs_c2_$g.log; exit 1; }
  tail -1 gpurun_out/gs_c2_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 g$g', d['ms_per_step'], r['frac'], d['frame_checksums']['match_n1'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gs -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 50 --warmup 2 --no-cpu-baseline > gpurun_out/prof_gs.log 2>&1 || exit 1
echo done
