#!/bin/bash
# Round 5: k_index1 with sc1 aggregate loads (no acquire fence) and one round trip for the chunk counts: the
# bucket / config-3 parity tests, the per-chunk stamps (probe build), then config 3 one launch vs two.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bucket or backward or ragged" > gpurun_out/r05_index1c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r05_index1c_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_index1c_tests.log | head; exit $rc; }
SHPL_LIB=sparse_pooling_amd/variants/lib_shplprobe.so timeout -k 10 200 python scripts/stamps_idx1.py || exit 1
for r in 1 2; do
  bash scripts/ab_kernels.sh r05_index1c_$r "--config 3 --steps 200" "k_index1|k_count|k_compact" \
    one=sparse_pooling_amd/libshpl.so two=sparse_pooling_amd/variants/lib_shplindex10.so || exit 1
done
echo done
