#!/bin/bash
# Round 5: the whole GPU suite + smoke on the cleaned wide conv, then the RetinaNet conv line with its
# cpu_baseline (the oracle conv at 512 -> 256 channels on one band of rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05_smoke.log
timeout -k 10 400 python bench.py --workload conv --config 6 --dtype bf16 > gpurun_out/r05_bench_conv_c6_bf16.log 2>&1 || { tail -5 gpurun_out/r05_bench_conv_c6_bf16.log; exit 1; }
grep '^{' gpurun_out/r05_bench_conv_c6_bf16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['kernel_ms'], d['cpu_baseline'], (d['frame_checksums'] or {}).get('match_n1'))"
echo done
