#!/bin/bash
# Round 6: the bf16 training backward's image gradient on the side stream beside the weight gradient (zero rows
# + pull after the input gradient) against its zero rows beside the input gradient (the default); the side-stream
# test first. Interleaved bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r06_beside; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_grad.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "side_stream or reuse" > $o/tests.log 2>&1
rc=$?; tail -1 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $o/tests.log | head; exit $rc; }
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline "$@" > $o/bench_$n.log 2>&1 || { tail -5 $o/bench_$n.log; exit 1; }
  grep '^{' $o/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['ms_per_step'], r['frac'])"
}
for k in 1 2 3; do
  run dgrad_$k --img-beside dgrad
  run wgrad_$k --img-beside wgrad
done
echo done
