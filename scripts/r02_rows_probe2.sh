cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t7; export TMPDIR=/tmp
for v in default rprobe1 rprobe2; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps 10 > gpurun_out/t7/conv_$v.log 2>&1 || { tail -5 gpurun_out/t7/conv_$v.log; exit 1; }
  grep '^{' gpurun_out/t7/conv_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v fused', r.get('kernel_ms'), 'dense', d['unfused']['conv_ms'])"
  timeout -k 10 200 python scripts/time_conv_parts.py > gpurun_out/t7/parts_$v.log 2>&1 || { tail -5 gpurun_out/t7/parts_$v.log; exit 1; }
  tail -1 gpurun_out/t7/parts_$v.log
done
