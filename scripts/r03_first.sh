#!/bin/bash
# Round 3, first GPU pass: the whole GPU suite, smoke, the default bench (both
# CPU-baseline legs), the 8-rank config-4 rehearsal on the one device (gloo
# control plane, 8 frames per rank), and a kernel trace of config 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/bench.log | cut -c1-400
SHPL_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --steps 20 > gpurun_out/rehearse_n8.log 2>&1 || { tail -20 gpurun_out/rehearse_n8.log; exit 1; }
grep '^{' gpurun_out/rehearse_n8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=8 gloo', d['value'], d['ms_per_step'], d['frame_checksums'], d['comm']['world_size'], d['comm']['backend'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit 1
grep '^{' gpurun_out/prof_c3.log | cut -c1-300
echo done
