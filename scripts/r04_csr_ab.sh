#!/bin/bash
# The CSR builder of the conv and training workloads (their CSR is on the critical path, not beside a
# stream): the per-frame sort (auto at 64 frames) against the segmented one, bench line + kernel trace each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=sparse_pooling_amd/libshpl.so
P="k_csr|k_zero32|k_conv_rows|k_pool_runs|k_occ"
bash scripts/ab_args.sh r04_csrconv "--workload conv --dtype bf16" "$P" "auto=$N" "seg=$N|--csr-path segment" "auto2=$N" "seg2=$N|--csr-path segment" || exit 1
bash scripts/ab_args.sh r04_csrtrain "--workload conv --train --dtype bf16 --steps 10" "$P" "auto=$N" "seg=$N|--csr-path segment" || exit 1
