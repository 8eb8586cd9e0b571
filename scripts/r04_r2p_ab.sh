#!/bin/bash
# (The kernel was removed from the sources after this measurement; commit history has it.)
# Config 3's pull pairs on persistent, software-pipelined waves (k_rows2p, SHPL_ROWS2P) against k_rows2:
# parity (the pipeline / ops / checksum-oracle tests), then the bench line and kernel trace of each, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=sparse_pooling_amd/variants/libshpl_r2.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_checksums_oracle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_r2p_tests.log 2>&1 || { tail -30 gpurun_out/r04_r2p_tests.log; exit 1; }
tail -1 gpurun_out/r04_r2p_tests.log
bash scripts/ab_kernels.sh r04_r2p "--config 3 --steps 200" "k_count|k_compact|k_bsort2|k_rows2" rows2=$V r2p=$N rows2b=$V r2pb=$N
