#!/bin/bash
# Round 5: config 6's split step with the index chain on the high-priority stream the step runs on (only the
# copy forked: one cross-stream hop per step) against the chain on a stream of its own; split tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "split" > gpurun_out/r05_c6chain_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r05_c6chain_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_c6chain_tests.log | head; exit $rc; }
L=sparse_pooling_amd/libshpl.so
for r in 1 2; do
  bash scripts/ab_args.sh r05_c6chain_$r "--config 6" "k_once|k_dense|k_csr_frame" \
    "current=$L|--split-chain current" "stream=$L|--split-chain stream" || exit 1
done
echo done
