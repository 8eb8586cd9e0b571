#!/bin/bash
# Round 3: the raw-scan step with the streaming pass started at different points of the index chain
# (bench.py --dense-after start|velo|bev|csr), f32 BEV input; the frames parity tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/da; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "velo or frames or kitti" -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/da/tests.log 2>&1; rc=$?; tail -2 gpurun_out/da/tests.log; [ $rc -eq 0 ] || exit $rc
for a in ${ORDER:-start velo bev csr start velo bev csr}; do
  timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline --maps-form ${FORM:-bev_input} --dense-after $a > gpurun_out/da/fr_$a.log 2>&1 || { tail -5 gpurun_out/da/fr_$a.log; exit 1; }
  grep '^{' gpurun_out/da/fr_$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_frac'], {k: round(v, 3) for k, v in d['stages_ms'].items()}, d['frame_checksums']['match_n1'])"
done
echo done
