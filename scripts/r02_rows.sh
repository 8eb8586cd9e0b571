#!/bin/bash
# Row-streaming bf16 conv (k_conv_rows): its parity tests, then the conv workload
# (config 2 + fused conv, bf16) with it and with the tiled kernel (variants/norows.so,
# built with SHPL_CONV_ROWS=0), then a kernel trace of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${TESTSEL:+-k "$TESTSEL"} > gpurun_out/rows_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/rows_tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-default norows}; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 300 python bench.py --workload conv --dtype bf16 ${BENCH_ARGS} --no-cpu-baseline > gpurun_out/rows_$v.log 2>&1 || { tail -5 gpurun_out/rows_$v.log; exit 1; }
  tail -1 gpurun_out/rows_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['frac'], r.get('kernel_ms'), d.get('unfused'))"
done
unset SHPL_LIB
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rows -o run --output-format csv -- \
    python3 bench.py --workload conv --dtype bf16 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_rows.log 2>&1 || exit 1
  find gpurun_out/prof_rows -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/rows_kernel_stats.csv
fi
echo done
