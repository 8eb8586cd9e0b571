#!/bin/bash
# Round 3: config 3 A/B of library variants (SHPL_LIB=variants/<v>.so) after the bucket parity subset.
# VARIANTS: space-separated list (default = the default library only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTS:-bucket or backward}" > gpurun_out/c3ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/c3ab_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/c3ab_tests.log | head -30; exit $rc; }
for v in ${VARIANTS:-default} ${VARIANTS:-default}; do
  # x-<name>: the default library with bench flag --no-<name>; y-<name>: with --<name>;
  # <lib>+<flag>: variants/<lib>.so with --<flag>
  x=""; lib="$v"
  case "$v" in x-*) x="--no-${v#x-}"; lib=default;; y-*) x="--${v#y-}"; lib=default;; *+*) x="--${v#*+}"; lib="${v%%+*}";; esac
  if [ "$lib" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$lib.so; fi
  timeout -k 10 300 python bench.py --config 3 --steps 200 --no-cpu-baseline $x $BENCH_EXTRA > gpurun_out/c3ab_$v.log 2>&1 || { tail -5 gpurun_out/c3ab_$v.log; exit 1; }
  tail -1 gpurun_out/c3ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['frac'], r.get('k_sparse_ms'), r.get('backward_ms'), d['frame_checksums']['match_n1'])"
done
unset SHPL_LIB
if [ -n "$FRAMES" ]; then  # the raw-scan step with the BEV maps in each form
  for m in f64 bev_input f64 bev_input; do
    timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline --maps-form $m > gpurun_out/fr_$m.log 2>&1 || { tail -5 gpurun_out/fr_$m.log; exit 1; }
    tail -1 gpurun_out/fr_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('frames $m', d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_frac'], d['stages_ms']['k_dense_ms'], d['frame_checksums']['match_n1'])"
  done
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3ab -o run --output-format csv -- \
    python3 bench.py --config 3 --steps 50 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3ab.log 2>&1 || exit 1
fi
if [ -n "$PROF2" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3ab2 -o run --output-format csv -- \
    python3 bench.py --config 3 --steps 50 --warmup 2 --no-cpu-baseline $PROF2 > gpurun_out/prof_c3ab2.log 2>&1 || exit 1
fi
echo done
