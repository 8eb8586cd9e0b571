# k_pool_runs with each entry's row loads issued beside the next entry's index words, vs the previous build
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pr; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py tests/test_gpu_rows_fuzz.py -k "bf16 or rows or pooled" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pr/tests.log 2>&1; rc=$?; tail -2 gpurun_out/pr/tests.log; [ $rc -eq 0 ] || exit $rc
for v in new prv_old new prv_old; do
  if [ "$v" = new ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps 20 > gpurun_out/pr/conv_$v.log 2>&1 || { tail -3 gpurun_out/pr/conv_$v.log; exit 1; }
  grep '^{' gpurun_out/pr/conv_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['unfused']['bitwise_equal'], d['frame_checksums']['match_n1'])"
done
for v in new prv_old; do
  if [ "$v" = new ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pr/prof_$v -o run --output-format csv -- python3 bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/pr/p_$v.log 2>&1 || exit 1
done
echo done
