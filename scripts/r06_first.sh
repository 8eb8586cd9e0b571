#!/bin/bash
# Round 6, first GPU pass: the new robustness tests (k_index1 dirty words / forced give-up, the inference BN
# scale under graph-replayed training, config 4 at 8 ranks on one device), then the config-3 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 450 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_parity.py::test_index1_barrier_give_up_and_dirty_words" \
  "tests/test_gpu_conv.py::test_inference_scale_follows_graph_replayed_training" \
  "tests/test_gpu_conv.py::test_batch_norm_training_vs_oracle" \
  "tests/test_gpu_parity.py::test_pipeline_backward_matches_oracle" \
  "tests/test_gpu_dist.py::test_config4_eight_ranks_on_one_device_matches_stored_n1_table" \
  > gpurun_out/r06_first_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_first_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r06_first_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --config 3 --steps 200 --no-cpu-baseline > gpurun_out/r06_bench_c3.log 2>&1 || { tail -5 gpurun_out/r06_bench_c3.log; exit 1; }
grep '^{' gpurun_out/r06_bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c3', d['ms_per_step'], r['frac'], (d.get('frame_checksums') or {}).get('match_n1'))"
