#!/bin/bash
# Round 5: the training step's side-stream backward work (FusionConv.IMG_ZERO_SIDE: the image gradient's zero
# rows; WGRAD_SIDE: the weight gradient) against one stream: the bitwise test, then the bf16 training line per
# setting, alternating, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_grad.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_wside_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_wside_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_wside_tests.log | head; exit $rc; }
for r in 1 2; do
  for v in zero none wgrad; do
    case $v in
      zero) extra="--img-zero-side on --wgrad-side off";;
      none) extra="--img-zero-side off --wgrad-side off";;
      wgrad) extra="--img-zero-side off --wgrad-side on";;
    esac
    timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline $extra > gpurun_out/r05_wside_$v.log 2>&1 || { tail -5 gpurun_out/r05_wside_$v.log; exit 1; }
    grep '^{' gpurun_out/r05_wside_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['fwd_ms'], d['bwd_ms'], d['roofline']['frac'])"
  done
done
echo done
