#!/bin/bash
# Round 5: config 6 split pipeline (parity + A/B + kernel trace) and the RetinaNet conv shape on the existing kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split" tests/test_gpu_conv.py::test_retinanet_fusion_conv_shape -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_c6_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_c6_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_c6_tests.log | head -20; exit $rc; }
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], (d.get('frame_checksums') or {}).get('match_n1'), r.get('kernel_ms'), r.get('eager_brackets_ms'))"; }
for v in on off on off; do
  timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --split $v > gpurun_out/r05_c6_split_$v.log 2>&1 || { tail -5 gpurun_out/r05_c6_split_$v.log; exit 1; }
  line gpurun_out/r05_c6_split_$v.log c6_split_$v
done
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --split on --no-graph > gpurun_out/r05_c6_split_nograph.log 2>&1 || exit 1
line gpurun_out/r05_c6_split_nograph.log c6_split_nograph
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_c6_split -o run --output-format csv -- \
  python3 bench.py --config 6 --no-cpu-baseline --steps 10 --split on > gpurun_out/r05_prof_c6_split.log 2>&1 || { tail -5 gpurun_out/r05_prof_c6_split.log; exit 1; }
for dt in bf16 f32; do
  timeout -k 10 400 python bench.py --workload conv --config 6 --dtype $dt --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05_conv_c6_$dt.log 2>&1 || { tail -5 gpurun_out/r05_conv_c6_$dt.log; exit 1; }
  line gpurun_out/r05_conv_c6_$dt.log conv_c6_$dt
done
echo done
