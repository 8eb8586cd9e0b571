#!/bin/bash
# Round 6: which launch the forward pass-through copies ride at config 3 (each chain launch's
# length set by its bytes) -- both on the index launch (shipped), the cell copy on the CSR launch, the pixel copy
# there, both there: the rider tests, then the bench line + kernel trace of each placement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "ride_either or barrier" > gpurun_out/r06_riders_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_riders_tests.log; [ $rc -eq 0 ] || exit $rc
N=sparse_pooling_amd/libshpl.so
bash scripts/ab_args.sh r06_riders "--config 3 --steps 200" "k_index1|k_bsort2|k_rows2" \
  "ii=$N|" "ci=$N|--copy-at csr,index" "ic=$N|--copy-at index,csr" "cc=$N|--copy-at csr,csr" "ii2=$N|" "ci2=$N|--copy-at csr,index"
