#!/bin/bash
# Config 3: parity of the bucketed step on the new library, then the A/B against the previous one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_c3_tests.log 2>&1 || { tail -30 gpurun_out/r04_c3_tests.log; exit 1; }
tail -1 gpurun_out/r04_c3_tests.log
bash scripts/ab_kernels.sh "$@"
