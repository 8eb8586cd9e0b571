#!/bin/bash
# Round 5: run heads in the bucket CSRs (shpl_csr.heads: each destination's first entries read in the
# round trip of its key_range by the row-keyed pulls): the bucket / config-3 parity tests and the ABI, then
# config 3 with 8 (default), 0, 4 and 16 heads per destination, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "bucket or backward or ragged" > gpurun_out/r05_heads_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r05_heads_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_heads_tests.log | head; exit $rc; }
L=sparse_pooling_amd/libshpl.so
for r in 1 2; do
  bash scripts/ab_args.sh r05_heads_$r "--config 3 --steps 200" "k_rows2|k_bsort2" \
    "h8=$L|--head-k 8" "h0=$L|--head-k 0" "h4=$L|--head-k 4" "h16=$L|--head-k 16" || exit 1
done
echo done
