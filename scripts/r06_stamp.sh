#!/bin/bash
# Round 6: stamp profiles/traffic.json from the PMC passes scripts/r06_final2.sh left under gpurun_out/ (run here,
# after the GPU call): each entry is bound to the lib_sha256 its profiled bench printed. Anchors: the kernel
# launched once per step (k_count; k_index1 for the bucketed config-3 step; k_bev_frame for the raw-scan steps,
# whose velodyne stage launches k_count too -- round 5 stamped those two with k_count, halving them).
set -e
cd "$(dirname "$0")/.."
python3 scripts/traffic.py step config2_F64 c2f64
python3 scripts/traffic.py step config2_F8 c2f8
python3 scripts/traffic.py step config3_F4 c3f4 all k_index1
python3 scripts/traffic.py step config5_F64 c5f64
python3 scripts/traffic.py step frames_F64 frf64 layer k_bev_frame
python3 scripts/traffic.py step frames_bev_input_F64 frbev layer k_bev_frame
python3 scripts/traffic.py step train_bf16_F64 trbf16 all
python3 scripts/traffic.py step config6_F64 c6f64
python3 scripts/traffic.py conv_bf16_F64
python3 scripts/traffic.py conv_f32_F64
python3 scripts/traffic.py conv_c6_bf16_F64
