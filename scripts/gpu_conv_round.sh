#!/bin/bash
# Round-end evidence for the conv workloads: the bf16 training bench line, the
# rocprof kernel stats of the conv / conv-training benches (f32, bf16) and the
# PMC passes of the forward conv (gpu_conv_prof.sh). Each GPU step has its own
# time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > gpurun_out/bench_conv_train_bf16.log 2>&1 || exit $?
echo "train bf16 ok"
for DT in f32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_conv_train_$DT -o run --output-format csv -- \
    python3 bench.py --workload conv --train --dtype $DT --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/prof_conv_train_$DT.log 2>&1 || exit $?
  echo "train $DT prof ok"
  DT=$DT bash scripts/gpu_conv_prof.sh || exit $?
done
echo all done
