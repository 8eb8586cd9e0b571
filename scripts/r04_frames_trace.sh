#!/bin/bash
# Raw-scan step timeline: a kernel trace of bench --workload frames (bev_input maps), and of k_dense alone
# (--dense-after csr: the streaming pass after the chain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_frames
export TMPDIR=/tmp
for v in "beside|" "after|--dense-after csr"; do
  n=${v%%|*}; a=${v#*|}
  timeout -k 10 300 python bench.py --workload frames --maps-form bev_input --steps 10 --no-cpu-baseline $a > gpurun_out/r04_frames/bench_$n.log 2>&1 || { tail -5 gpurun_out/r04_frames/bench_$n.log; exit 1; }
  grep '^{' gpurun_out/r04_frames/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04_frames/prof_$n -o run --output-format csv -- \
    python3 bench.py --workload frames --maps-form bev_input --steps 10 --no-cpu-baseline $a > gpurun_out/r04_frames/prof_$n.log 2>&1 || { tail -5 gpurun_out/r04_frames/prof_$n.log; exit 1; }
done
echo done
