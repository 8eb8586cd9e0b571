cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fin; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fin/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fin/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || { tail gpurun_out/fin/smoke.log; exit 1; }
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/fin/bench.log 2>&1 || { tail -5 gpurun_out/fin/bench.log; exit 1; }
grep '^{' gpurun_out/fin/bench.log | cut -c1-200
export SHPL_DIST_BACKEND=gloo
for w in "" "--workload conv --dtype bf16" "--workload conv --train --dtype bf16"; do
  timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 $w > gpurun_out/fin/n2.log 2>&1 || { tail -20 gpurun_out/fin/n2.log; exit 1; }
  grep '^{' gpurun_out/fin/n2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2 [$w]', d['n_gpus'], d['value'], d['ms_per_step'], (d.get('frame_checksums') or {}).get('match_n1'))"
done
echo done
