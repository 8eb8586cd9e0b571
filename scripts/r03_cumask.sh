#!/bin/bash
# Round 3: the raw-scan step with the index chain on a CU-masked stream (bench --chain-cus K --cu-layout L
# [--dense-excl]), f32 BEV input. (The bench flags were removed after this A/B: profiles/r03_cumask_ab/summary.log.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cm; export TMPDIR=/tmp
i=0
while read -r name flags; do
  [ -z "$name" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py --workload frames --steps 20 --no-cpu-baseline --maps-form bev_input $flags > gpurun_out/cm/fr_$i.log 2>&1 || { tail -5 gpurun_out/cm/fr_$i.log; exit 1; }
  grep '^{' gpurun_out/cm/fr_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], d['roofline']['frac'], {k: round(v, 3) for k, v in d['stages_ms'].items()}, d['frame_checksums']['match_n1'])"
done <<'LIST'
default
s32 --chain-cus 32
s32x --chain-cus 32 --dense-excl
l32 --chain-cus 32 --cu-layout lo
l32x --chain-cus 32 --cu-layout lo --dense-excl
s64 --chain-cus 64
s64x --chain-cus 64 --dense-excl
s16x --chain-cus 16 --dense-excl
default
s32x --chain-cus 32 --dense-excl
LIST
echo done
