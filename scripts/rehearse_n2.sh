#!/bin/bash
# Rehearsal of bench.py's N>1 path on a one-GPU box: 2 ranks on the same GPU
# over gloo (SHPL_DIST_BACKEND=gloo); the driver's scaling runs use RCCL with
# one rank per GPU. Each run has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SHPL_DIST_BACKEND=gloo
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
i=0
for w in "--steps 5 --warmup 2" "--config 3 --steps 5 --warmup 2" "--config 5 --steps 3 --warmup 1" \
         "--workload frames --steps 3 --warmup 1" "--workload conv --steps 3 --warmup 1" \
         "--workload conv --train --steps 3 --warmup 1"; do
  i=$((i+1))
  timeout -k 10 300 $R --master-port $((29500 + i)) bench.py --gpus 2 $w > gpurun_out/n2_$i.log 2>&1
  rc=$?; echo "[$w] rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/n2_$i.log; exit $rc; }
  grep '^{' gpurun_out/n2_$i.log | cut -c1-220
done
