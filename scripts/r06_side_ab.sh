#!/bin/bash
# Round 6: with the input gradient's pooled map stored at occupied cells only, the side-stream placements of the
# bf16 training backward again (weight gradient / image-gradient zero rows beside the input gradient), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06_side
export TMPDIR=/tmp
o=gpurun_out/r06_side
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline "$@" > $o/bench_$n.log 2>&1 || { tail -5 $o/bench_$n.log; exit 1; }
  grep '^{' $o/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', d['ms_per_step'], r['frac'])"
}
for k in 1 2; do
  run base$k
  run wside$k --wgrad-side on
  run nozero$k --img-zero-side off
  run both$k --wgrad-side on --img-zero-side off
done
echo done
