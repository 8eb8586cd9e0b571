#!/bin/bash
# The frame CSR sort over several workgroups per frame (k_csr_frame split, default: by batch size) against one
# workgroup per frame (SHPL_CSR_SPLIT=1): parity, then the conv, training and config-2 steps. Measured and
# dropped (profiles/r04_split_ab.log); the split form was reverted.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=sparse_pooling_amd/variants/libshpl_split1.so
N=sparse_pooling_amd/libshpl.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checksums_oracle.py tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_split_tests.log 2>&1 || { tail -30 gpurun_out/r04_split_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04_split_tests.log)"
bash scripts/ab_args.sh r04_split_conv "--workload conv --dtype bf16" "k_csr_frame|k_conv_rows<4, 2" "one=$O" "split=$N" "one2=$O" "split2=$N" || exit 1
bash scripts/ab_args.sh r04_split_train "--workload conv --train --dtype bf16 --steps 10" "k_csr_frame|k_conv_rows<4, 2" "one=$O" "split=$N" || exit 1
bash scripts/ab_args.sh r04_split_c2 "--steps 20" "k_csr_frame|k_dense" "one=$O" "split=$N" "one2=$O" "split2=$N" || exit 1
