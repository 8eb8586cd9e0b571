#!/bin/bash
# Round 5: k_conv_wide halo DMAs nontemporal (weights kept in L2), with LDS-DMA weights and with register A; parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base hnt aregnt; do
  lib=""; [ $v != base ] && lib=sparse_pooling_amd/variants/lib_$v.so
  SHPL_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -k "wide or retinanet" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_wide6_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -1 gpurun_out/r05_wide6_tests_$v.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_wide6_tests_$v.log | head -20; exit $rc; }
done
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; u=d['unfused']; print('$2', d['ms_per_step'], r['frac'], 'fused', r.get('kernel_ms'), 'conv_only', u['conv_ms'])"; }
for rep in 1 2 3; do
for v in base hnt aregnt; do
  lib=""; [ $v != base ] && lib=sparse_pooling_amd/variants/lib_$v.so
  SHPL_LIB=$lib timeout -k 10 300 python bench.py --workload conv --config 6 --dtype bf16 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r05_wide_ab6_$v.log 2>&1 || { tail -5 gpurun_out/r05_wide_ab6_$v.log; exit 1; }
  line gpurun_out/r05_wide_ab6_$v.log $v
done
done
echo done
