cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t15; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t15/tests.log 2>&1; rc=$?; tail -8 gpurun_out/t15/tests.log; exit $rc
