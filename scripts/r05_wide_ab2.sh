#!/bin/bash
# Round 5: k_conv_wide one wave per SIMD (AGPR accumulators, default) vs two (SHPL_WIDE_WAVES=8), + probes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -k "wide or retinanet" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_wide4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_wide4_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_wide4_tests.log | head -20; exit $rc; }
SHPL_LIB=sparse_pooling_amd/variants/lib_wide8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -k "wide or retinanet" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_wide8_tests.log 2>&1
rc=$?; echo "tests8 rc=$rc"; tail -2 gpurun_out/r05_wide8_tests.log; [ $rc -eq 0 ] || exit $rc
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; u=d['unfused']; print('$2', d['ms_per_step'], r['frac'], 'fused', r.get('kernel_ms'), 'conv_only', u['conv_ms'])"; }
for rep in 1 2; do
for v in base wide8 wide4p1 wide4p3; do
  lib=""; [ $v != base ] && lib=sparse_pooling_amd/variants/lib_$v.so
  SHPL_LIB=$lib timeout -k 10 300 python bench.py --workload conv --config 6 --dtype bf16 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r05_wide_ab2_$v.log 2>&1 || { tail -5 gpurun_out/r05_wide_ab2_$v.log; exit 1; }
  line gpurun_out/r05_wide_ab2_$v.log $v
done
done
echo done
