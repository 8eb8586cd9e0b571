#!/bin/bash
# Round 5: k_conv_wide A/B (counted vmcnt vs vmcnt(0)) and timing probes (wrong results), RetinaNet shape, bf16;
# then one SQ PMC pass of the base kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; u=d['unfused']; print('$2', d['ms_per_step'], r['frac'], 'fused', r.get('kernel_ms'), 'conv_only', u['conv_ms'])"; }
for rep in 1 2; do
for v in base shplwidevmcnt0 shplwideprobe1 shplwideprobe2 shplwideprobe3; do
  lib=""; [ $v != base ] && lib=sparse_pooling_amd/variants/lib_$v.so
  SHPL_LIB=$lib timeout -k 10 300 python bench.py --workload conv --config 6 --dtype bf16 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r05_wide_ab_$v.log 2>&1 || { tail -5 gpurun_out/r05_wide_ab_$v.log; exit 1; }
  line gpurun_out/r05_wide_ab_$v.log $v
done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "conv_wide" -d gpurun_out/r05_wide_pmc -o run --output-format csv -- \
  python3 bench.py --workload conv --config 6 --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/r05_wide_pmc.log 2>&1
echo "pmc rc=$?"
echo done
