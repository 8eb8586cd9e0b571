cd $GRAFT_REPO_ROOT
for v in default probe1 probe2 probe3; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --no-cpu-baseline --steps 10 > gpurun_out/probe_$v.log 2>&1 || { tail -5 gpurun_out/probe_$v.log; exit 1; }
  tail -1 gpurun_out/probe_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', r.get('kernel_ms'), d['unfused']['conv_ms'])"
done
