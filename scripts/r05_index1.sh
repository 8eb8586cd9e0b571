#!/bin/bash
# Round 5, VERDICT r04 item 2: the bucketed index build's two launches (k_count + k_compact, riders split
# between them) against ONE launch with a frame barrier inside (k_index1, both copies riding it). The config-3
# and bucket parity tests on the default library first, then the config-3 bench line + kernel trace per
# library, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "bucket or backward or ragged or checksum" > gpurun_out/r05_index1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_index1_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_index1_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_checksums_oracle.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_index1_cs.log 2>&1
rc=$?; echo "checksum tests rc=$rc"; tail -2 gpurun_out/r05_index1_cs.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  bash scripts/ab_kernels.sh r05_index1_$r "--config 3 --steps 200" "k_index1|k_count|k_compact|k_bsort2|k_rows2" \
    one=sparse_pooling_amd/libshpl.so two=sparse_pooling_amd/variants/lib_shplindex10.so || exit 1
done
echo done
