#!/bin/bash
# Round 5: k_bsort2's counting sort with a DPP scan and LDS-atomic peers (instead of ds_bpermute shuffles and
# 7 ballots per batch) against the previous commit's library, config 3, twice; the bucket parity tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bucket or backward or ragged or csr or path" > gpurun_out/r05_bsort_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r05_bsort_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_bsort_tests.log | head; exit $rc; }
for r in 1 2; do
  bash scripts/ab_kernels.sh r05_bsort_$r "--config 3 --steps 200" "k_index1|k_bsort2|k_rows2" \
    new=sparse_pooling_amd/libshpl.so old=sparse_pooling_amd/variants/lib_shplbs0.so || exit 1
done
echo done
