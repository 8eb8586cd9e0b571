#!/bin/bash
# Copies a gpu_full.sh run's summaries from gpurun_out/ (scratch) into
# profiles/ (tracked) under this round's names, and recomputes the PMC
# traffic of the default bench line (profiles/traffic.json).
cd "$(dirname "$0")/.."
R=${ROUND:-r01}
o=gpurun_out
cp $o/bench.log profiles/${R}_bench.log
cp $o/gpu_tests.log profiles/${R}_gpu_tests.log
cp $o/smoke.log profiles/${R}_smoke.log
cp $o/prof/run_kernel_stats.csv profiles/${R}_kernel_stats.csv
cp $o/bench_c3.log profiles/${R}_bench_config3.log
cp $o/bench_c5.log profiles/${R}_bench_config5.log
cp $o/bench_frames.log profiles/${R}_bench_frames.log
cp $o/bench_noov.log profiles/${R}_bench_no_overlap.log
cp $o/bench_conv.log profiles/${R}_bench_conv.log
cp $o/bench_conv_bf16.log profiles/${R}_bench_conv_bf16.log
cp $o/bench_conv_train.log profiles/${R}_bench_conv_train.log
for c in 3 5; do cp $o/prof_c$c/run_kernel_stats.csv profiles/${R}_config${c}_kernel_stats.csv; done
cp $o/prof_frames/run_kernel_stats.csv profiles/${R}_frames_kernel_stats.csv
python3 scripts/traffic.py config2_F64
mkdir -p profiles/${R}_pmc
for c in FETCH_SIZE WRITE_SIZE; do
  f=$(find $o/pmc_$c -name '*counter_collection.csv' | head -1); [ -n "$f" ] && cp "$f" profiles/${R}_pmc/$c.csv
done
