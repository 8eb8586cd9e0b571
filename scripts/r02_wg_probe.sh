cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t5; export TMPDIR=/tmp
for v in default wgprobe1; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python scripts/time_conv_parts.py > gpurun_out/t5/$v.log 2>&1 || { tail -5 gpurun_out/t5/$v.log; exit 1; }
  tail -1 gpurun_out/t5/$v.log
done
