#!/bin/bash
# The 16x16x32 row conv: conv parity, then the bf16 conv workload's per-frame checksum table rewritten (the
# outputs changed within the tolerance; copied to gpurun_out/ -- the box's profiles/ does not come back).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_m16_final_tests.log 2>&1 || { tail -30 gpurun_out/r04_m16_final_tests.log; exit 1; }
tail -1 gpurun_out/r04_m16_final_tests.log
timeout -k 10 400 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --write-checksums > gpurun_out/bench_conv_table.log 2>&1 || { tail -5 gpurun_out/bench_conv_table.log; exit 1; }
cp profiles/frame_checksums.json gpurun_out/frame_checksums_conv.json
timeout -k 10 400 python bench.py --workload conv --dtype bf16 --no-cpu-baseline > gpurun_out/bench_conv_check.log 2>&1 || { tail -5 gpurun_out/bench_conv_check.log; exit 1; }
grep '^{' gpurun_out/bench_conv_check.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('conv', d['ms_per_step'], d['roofline']['frac'], d['frame_checksums']['match_n1'])"
