#!/bin/bash
# Round 6 diagnosis: the bucket sort's failed-barrier checks (shipped) against none (SHPL_BSORT_CHECKS=0) and
# against the round-5 index chain (libshpl_r5idx): config-3 bench + kernel trace, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_kernels.sh r06_chk "--config 3 --steps 200" "k_index1|k_bsort2" r5idx=sparse_pooling_amd/variants/libshpl_r5idx.so \
  nochk=sparse_pooling_amd/variants/libshpl_nochk.so chk=sparse_pooling_amd/libshpl.so r5idxb=sparse_pooling_amd/variants/libshpl_r5idx.so \
  nochkb=sparse_pooling_amd/variants/libshpl_nochk.so chkb=sparse_pooling_amd/libshpl.so
