# A/B: the dense 1- and 2-chunk k_conv_rows forms at 3 waves per SIMD (variants/wpe3.so) against the default 2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wpe; export TMPDIR=/tmp
export SHPL_LIB=$PWD/sparse_pooling_amd/variants/wpe3.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -k "bf16 or rows" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/wpe/tests.log 2>&1; rc=$?; tail -3 gpurun_out/wpe/tests.log; [ $rc -eq 0 ] || exit $rc
for v in wpe3 default wpe3 default; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python scripts/time_conv_parts.py > gpurun_out/wpe/parts_$v.log 2>&1 || exit 1; echo "$v $(tail -1 gpurun_out/wpe/parts_$v.log | cut -c1-160)"
done
