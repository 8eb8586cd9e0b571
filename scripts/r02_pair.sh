cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t14; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "backward_matches_oracle or rows or csr" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t14/tests.log 2>&1; rc=$?; tail -3 gpurun_out/t14/tests.log; [ $rc -eq 0 ] || exit $rc
for a in "" "--no-pair" "" "--no-pair"; do
  timeout -k 10 300 python bench.py --config 3 --steps 50 --no-cpu-baseline $a > gpurun_out/t14/c3$a.log 2>&1 || exit 1
  grep '^{' gpurun_out/t14/c3$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$a]', d['ms_per_step'], d['roofline']['frac'], d['frame_checksums']['match_n1'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t14/prof -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/t14/prof.log 2>&1 || exit 1
echo ok
