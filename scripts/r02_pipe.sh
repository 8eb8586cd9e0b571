cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t8; export TMPDIR=/tmp
export SHPL_LIB=$PWD/sparse_pooling_amd/variants/pipe.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k "bf16" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t8/tests.log 2>&1; rc=$?; tail -5 gpurun_out/t8/tests.log; [ $rc -eq 0 ] || exit $rc
for v in pipe default; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps 10 > gpurun_out/t8/conv_$v.log 2>&1 || { tail -5 gpurun_out/t8/conv_$v.log; exit 1; }
  grep '^{' gpurun_out/t8/conv_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v fused', r.get('kernel_ms'), 'dense', d['unfused']['conv_ms'], d['unfused']['bitwise_equal'], d['frame_checksums']['match_n1'])"
done
