#!/bin/bash
# Round 5: shpl_pull_once variants at config 6 (split step, eager): zero blocks first, 32 / 64 rows per wave.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], (d.get('frame_checksums') or {}).get('match_n1'), r.get('kernel_ms'))"; }
for rep in 1 2; do
for v in base shploncezerofirst1 shploncerows32 shploncerows64; do
  lib=""; [ $v != base ] && lib=sparse_pooling_amd/variants/lib_$v.so
  SHPL_LIB=$lib timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --steps 40 > gpurun_out/r05_once_ab_$v.log 2>&1 || { tail -5 gpurun_out/r05_once_ab_$v.log; exit 1; }
  line gpurun_out/r05_once_ab_$v.log $v
done
done
echo done
