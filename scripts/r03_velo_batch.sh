#!/bin/bash
# Round 3: scan rows per thread of the velodyne compaction (SHPL_VELO_BATCH, variants/velo<b>.so) on the
# raw-scan step (f32 BEV input); the KITTI / raw-scan parity tests under each variant first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vb; export TMPDIR=/tmp
for v in ${VARIANTS:-velo2 velo4 velo8}; do
  SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "velo or frames or kitti" -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/vb/tests_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/vb/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in default ${VARIANTS:-velo2 velo4 velo8} default ${VARIANTS:-velo2 velo4 velo8}; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline --maps-form ${FORM:-bev_input} > gpurun_out/vb/fr_$v.log 2>&1 || { tail -5 gpurun_out/vb/fr_$v.log; exit 1; }
  grep '^{' gpurun_out/vb/fr_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_frac'], {k: round(v, 3) for k, v in d['stages_ms'].items()}, d['frame_checksums']['match_n1'])"
done
unset SHPL_LIB
for v in velo4; do  # the chain alone (streaming pass after the CSR)
  SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline --maps-form bev_input --dense-after csr > gpurun_out/vb/frcsr_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/vb/frcsr_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v alone', d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})"
done
echo done
