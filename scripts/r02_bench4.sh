cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t6; export TMPDIR=/tmp
for w in "--workload conv --train --dtype bf16" "--workload conv --train" "--workload conv --dtype bf16" "--workload frames"; do
  n=$(echo $w | tr -d ' -'); timeout -k 10 300 python bench.py $w --no-cpu-baseline > gpurun_out/t6/$n.log 2>&1 || { tail -5 gpurun_out/t6/$n.log; exit 1; }
  grep '^{' gpurun_out/t6/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:400])"
done
