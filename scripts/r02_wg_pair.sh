cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t13; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_gpu_conv.py -k "wgrad or pooled_stats or training" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t13/tests.log 2>&1; rc=$?; tail -3 gpurun_out/t13/tests.log; [ $rc -eq 0 ] || exit $rc
for v in default wgsingle default wgsingle; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python scripts/time_conv_parts.py > gpurun_out/t13/parts_$v.log 2>&1 || { tail -5 gpurun_out/t13/parts_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/t13/parts_$v.log)"
  timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > gpurun_out/t13/train_$v.log 2>&1 || exit 1; grep '^{' gpurun_out/t13/train_$v.log | cut -c180-260
done
