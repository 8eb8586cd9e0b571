cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t9; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t9/tests.log 2>&1; rc=$?; tail -12 gpurun_out/t9/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > gpurun_out/t9/train_bf16.log 2>&1 || exit 1; grep '^{' gpurun_out/t9/train_bf16.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t9/prof -o run --output-format csv -- python3 bench.py --workload conv --train --dtype bf16 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/t9/prof.log 2>&1 || exit 1
echo ok
