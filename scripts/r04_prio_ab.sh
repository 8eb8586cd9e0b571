#!/bin/bash
# Raw-scan step: which stream runs at high priority (the index chain: default; the streaming pass; both;
# neither), bench line and kernel trace each (f32 BEV input form).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=sparse_pooling_amd/libshpl.so
bash scripts/ab_args.sh r04_prio "--workload frames --maps-form bev_input --steps 10" "k_dense|k_sparse" "chain=$N|--stream-priority chain" "dense=$N|--stream-priority dense" "both=$N|--stream-priority both" "none=$N|--stream-priority none" "chain2=$N|--stream-priority chain" "dense2=$N|--stream-priority dense"
