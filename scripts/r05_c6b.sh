#!/bin/bash
# Round 5: config 6 split pipeline with shpl_pull_once (parity + A/B + traces), the RetinaNet conv test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_split_pipeline_matches_oracle tests/test_gpu_conv.py::test_retinanet_fusion_conv_shape tests/test_gpu_checksums_oracle.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_c6b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_c6b_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05_c6b_tests.log | head -20; exit $rc; }
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], (d.get('frame_checksums') or {}).get('match_n1'), r.get('kernel_ms'), r.get('eager_brackets_ms'))"; }
for a in "on" "on --no-graph" "on --split-pull rows --no-graph" "off" "on" "on --no-graph"; do
  n=$(echo $a | tr -d ' -')
  timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --split $a > gpurun_out/r05_c6b_$n.log 2>&1 || { tail -5 gpurun_out/r05_c6b_$n.log; exit 1; }
  line gpurun_out/r05_c6b_$n.log "$a"
done
for g in "" "--no-graph"; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_c6_once$g -o run --output-format csv -- \
  python3 bench.py --config 6 --no-cpu-baseline --steps 10 --split on $g > gpurun_out/r05_prof_c6_once$g.log 2>&1 || { tail -5 gpurun_out/r05_prof_c6_once$g.log; exit 1; }
done
echo done
