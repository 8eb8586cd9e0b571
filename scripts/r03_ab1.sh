#!/bin/bash
# Round 3 batch 2: the whole GPU suite on the default library (staged row pulls,
# branch-free pooled wgrad staging, LDS offsets for the spilling pooled conv form),
# config-3 A/B of the staged pull variants, the rebuilt 8-byte-store epilogue
# (SHPL_ROWS_EPI8) through the row-kernel fuzz tests, and the bf16 training step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for v in default old lds64 ppt2 nodma; do
  for r in 1 2; do
    if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
    timeout -k 10 300 python bench.py --config 3 --steps 100 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'), d['frame_checksums']['match_n1'])"
  done
done
unset SHPL_LIB
timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --steps 20 --no-cpu-baseline > gpurun_out/train_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/train_bf16.log | cut -c1-300
SHPL_LIB=$PWD/sparse_pooling_amd/variants/epi8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rows_fuzz.py tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/epi8_tests.log 2>&1
echo "epi8 tests rc=$?"; tail -15 gpurun_out/epi8_tests.log
echo done
