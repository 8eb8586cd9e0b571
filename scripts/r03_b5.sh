#!/bin/bash
# Round 3 batch 5: long-run / velodyne parity, raw-scan maps placement A/B, the bf16 conv and
# training steps after the epilogue change (fmax ReLU, no int16 max).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "long_run or velodyne or epilogue or rows" > gpurun_out/b5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/b5_tests.log; [ $rc -eq 0 ] || exit $rc
for m in stream chain stream chain; do
  timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline --maps-after $m > gpurun_out/fr_$m.log 2>&1 || { tail -5 gpurun_out/fr_$m.log; exit 1; }
  tail -1 gpurun_out/fr_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_frac'], d['stages_ms']['k_dense_ms'], d['frame_checksums']['match_n1'])"
done
timeout -k 10 300 python bench.py --workload conv --dtype bf16 --steps 20 --no-cpu-baseline > gpurun_out/conv_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/conv_bf16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('conv bf16', d['ms_per_step'], r['kernel_ms'], r['frac'], d['frame_checksums']['match_n1'], d['unfused']['bitwise_equal'])"
timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --steps 20 --no-cpu-baseline > gpurun_out/train_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/train_bf16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('train bf16', d['ms_per_step'], d['roofline']['frac'])"
echo done
