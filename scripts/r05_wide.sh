#!/bin/bash
# Round 5: the wide bf16 conv (k_conv_wide) -- parity vs the oracle, the RetinaNet conv bench line, a trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -k "wide or retinanet" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_wide_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_wide_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_wide_tests.log | head -20; exit $rc; }
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('kernel_ms'), r.get('hbm_frac'), d.get('unfused'))"; }
timeout -k 10 400 python bench.py --workload conv --config 6 --dtype bf16 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05_conv_c6_bf16_wide.log 2>&1 || { tail -5 gpurun_out/r05_conv_c6_bf16_wide.log; exit 1; }
line gpurun_out/r05_conv_c6_bf16_wide.log conv_c6_bf16
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_conv_c6 -o run --output-format csv -- \
  python3 bench.py --workload conv --config 6 --dtype bf16 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r05_prof_conv_c6.log 2>&1 || { tail -5 gpurun_out/r05_prof_conv_c6.log; exit 1; }
echo done
