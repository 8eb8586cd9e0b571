cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t16; export TMPDIR=/tmp
for F in 64 61 68 55 64; do
  timeout -k 10 200 python bench.py --workload conv --dtype bf16 --frames $F --steps 20 --no-cpu-baseline > gpurun_out/t16/f$F.log 2>&1 || { tail -3 gpurun_out/t16/f$F.log; exit 1; }
  grep '^{' gpurun_out/t16/f$F.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('F=$F rounds=%.2f'%(300*$F/2048), 'conv_ms', r['kernel_ms'], 'per_frame_us', round(1000*r['kernel_ms']/$F,2))"
done
