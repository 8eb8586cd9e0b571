# A/B: the next row's DMAs between this row's MFMAs (variants/dmai.so, SHPL_ROWS_DMAI=1, dense forms) vs default
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dmai; export TMPDIR=/tmp
export SHPL_LIB=$PWD/sparse_pooling_amd/variants/dmai.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -k "bf16 or rows" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/dmai/tests.log 2>&1; rc=$?; tail -3 gpurun_out/dmai/tests.log; [ $rc -eq 0 ] || exit $rc
for v in dmai default dmai default; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps 20 > gpurun_out/dmai/conv_$v.log 2>&1 || { tail -3 gpurun_out/dmai/conv_$v.log; exit 1; }
  grep '^{' gpurun_out/dmai/conv_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v fused', d['roofline']['kernel_ms'], 'dense', d['unfused']['conv_ms'], d['unfused']['bitwise_equal'], d['frame_checksums']['match_n1'])"
  timeout -k 10 200 python scripts/time_conv_parts.py > gpurun_out/dmai/parts_$v.log 2>&1 || exit 1; echo "$v $(tail -1 gpurun_out/dmai/parts_$v.log | cut -c1-120)"
done
