#!/bin/bash
# The row-keyed pipeline (--rows: bucketed index, one k_rows2 launch per pull pair) against the default
# k_dense + k_sparse path at 64 frames: config 6 (the RetinaNet P2 shape) and config 2, bench line and kernel
# trace each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=sparse_pooling_amd/libshpl.so
bash scripts/ab_args.sh r04_rows6 "--config 6" "k_dense|k_sparse|k_rows2|k_count|k_compact|k_bsort2|k_csr_frame" "dense=$N" "rows=$N|--rows" "dense2=$N" "rows2=$N|--rows" || exit 1
bash scripts/ab_args.sh r04_rows2 "--config 2" "k_dense|k_sparse|k_rows2|k_count|k_compact|k_bsort2|k_csr_frame" "dense=$N" "rows=$N|--rows" || exit 1
