cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for path in segment frame; do for cfg in 3 2; do
  SHPL_CSR_PATH=$path timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_${path}_$cfg.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_${path}_$cfg.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$path', 'cfg$cfg', j['value'], j['ms_per_step'], j['roofline']['frac'])"
done; done
