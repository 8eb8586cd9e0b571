#!/bin/bash
# Round 5: k_index1 variants on config 3 (bench line + kernel trace each): the default (SHPL_IDX1_RIDERS 240:
# 60 rider workgroups per copy and frame), 120 and 60 riders per copy over the batch, the two-launch form; and
# the default without riders (--no-riders: the copies as k_dense beside, k_index1's own duration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bucket or backward" > gpurun_out/r05_index1b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r05_index1b_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  bash scripts/ab_kernels.sh r05_index1b_$r "--config 3 --steps 200" "k_index1|k_count|k_compact" \
    r240=sparse_pooling_amd/libshpl.so r120=sparse_pooling_amd/variants/lib_shplr120.so \
    r60=sparse_pooling_amd/variants/lib_shplr60.so wpe8=sparse_pooling_amd/variants/lib_shplwpe8.so two=sparse_pooling_amd/variants/lib_shplindex10.so || exit 1
done
bash scripts/ab_kernels.sh r05_index1b_nr "--config 3 --steps 200 --no-riders" "k_index1|k_dense" \
  norider=sparse_pooling_amd/libshpl.so || exit 1
echo done
