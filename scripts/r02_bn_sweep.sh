# BatchNorm stream kernels (bf16 training step): rows per iteration / rows per thread variants, kernel times
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/bn; export TMPDIR=/tmp
for v in default bn_u8 bn_rpt16 bn_u8rpt16 bn_rpt4; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bn/prof_$v -o run --output-format csv -- \
    python3 bench.py --workload conv --train --dtype bf16 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bn/p_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/bn/p_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v step', d['ms_per_step'])"
done
echo done
