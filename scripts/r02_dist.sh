#!/bin/bash
# Config-4 evidence on the one-GPU box: the new parity cases, N=1 runs of every
# workload storing their per-frame checksums (profiles/frame_checksums.json), then
# the 2-rank rehearsal (gloo control plane, both ranks on the one GPU) through
# bench.py's own --gpus self-launch, whose checksums must match N=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -k "dist or partition or backward" \
  -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/dist_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/dist_tests.log; [ $rc -le 1 ] || exit $rc
i=0
for w in "" "--config 3" "--config 5" "--workload frames" "--workload conv" "--workload conv --dtype bf16"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --write-checksums $w > gpurun_out/n1_$i.log 2>&1 || { tail -5 gpurun_out/n1_$i.log; exit 1; }
  grep '^{' gpurun_out/n1_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=1 [$w]', d['value'], d['ms_per_step'], d['frame_checksums'])"
done
cp profiles/frame_checksums.json gpurun_out/frame_checksums.json
export SHPL_DIST_BACKEND=gloo
i=0
for w in "" "--config 3" "--config 5" "--workload frames" "--workload conv" "--workload conv --dtype bf16" "--workload conv --train"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 $w > gpurun_out/n2_$i.log 2>&1 || { tail -20 gpurun_out/n2_$i.log; exit 1; }
  grep '^{' gpurun_out/n2_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2 [$w]', d['value'], d['ms_per_step'], d['scaling'], d.get('frame_checksums'))"
done
for f in 8 16 32; do
  timeout -k 10 300 python bench.py --frames $f --steps 50 --no-cpu-baseline > gpurun_out/bench_f$f.log 2>&1 || exit 1
  grep '^{' gpurun_out/bench_f$f.log | cut -c1-200
done
