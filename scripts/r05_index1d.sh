#!/bin/bash
# Round 5: k_index1's riders: the launch without them (--no-riders: k_index1 alone, the copies as k_dense),
# and 16 instead of 8 pieces in flight per rider thread (SHPL_CP_BATCH=16), config 3, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  bash scripts/ab_kernels.sh r05_index1d_$r "--config 3 --steps 200" "k_index1|k_dense" \
    base=sparse_pooling_amd/libshpl.so cpb16=sparse_pooling_amd/variants/lib_shplcpb16.so || exit 1
  bash scripts/ab_kernels.sh r05_index1d_nr_$r "--config 3 --steps 200 --no-riders" "k_index1|k_dense" \
    norider=sparse_pooling_amd/libshpl.so || exit 1
done
echo done
