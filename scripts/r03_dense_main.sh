#!/bin/bash
# Round 3: configs 2 / 5 (and the N=8 rank shape) with the streaming half on the main queue and the index
# chain on the side one (bench --dense-main 1) vs the round-2 layout; the pipeline parity tests first. (The flag was removed after this A/B: profiles/r03_dense_main_ab/summary.log.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dm; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "pipeline or overlap or dist or bench or backward" > gpurun_out/dm/tests.log 2>&1; rc=$?; tail -1 gpurun_out/dm/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for c in "c2:" "c2f8:--frames 8" "c5:--config 5"; do
    name=${c%%:*}; flags=${c#*:}
    for dm in 0 1; do
      timeout -k 10 300 python bench.py $flags --no-cpu-baseline --no-pool-report --dense-main $dm > gpurun_out/dm/${name}_$dm.log 2>&1 || { tail -5 gpurun_out/dm/${name}_$dm.log; exit 1; }
      grep '^{' gpurun_out/dm/${name}_$dm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name dm=$dm', d['ms_per_step'], r['frac'], r.get('kernel_ms'), d['frame_checksums']['match_n1'])"
    done
  done
done
echo done
