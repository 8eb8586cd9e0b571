#!/bin/bash
# Round 3: the paired-wave weight gradient (SHPL_WG_PAIR, input tiles 2p / 2p+1 share each staged G row) vs one
# wave per input tile (variants/nopair.so): the wgrad / training tests, per-conv times with the wgrad digest
# (bitwise A/B), and the bf16 training bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wgp; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_grad.py tests/test_gpu_conv.py tests/test_gpu_rows_fuzz.py \
  -k "wgrad or training or pooled or fuzz" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/wgp/tests.log 2>&1; rc=$?; tail -3 gpurun_out/wgp/tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-default nopair default nopair}; do
  if [ "$v" = default ]; then unset SHPL_LIB; else export SHPL_LIB=$PWD/sparse_pooling_amd/variants/$v.so; fi
  timeout -k 10 200 python scripts/time_conv_parts.py > gpurun_out/wgp/parts_$v.log 2>&1 || { tail -5 gpurun_out/wgp/parts_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/wgp/parts_$v.log)"
  timeout -k 10 300 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > gpurun_out/wgp/train_$v.log 2>&1 || { tail -5 gpurun_out/wgp/train_$v.log; exit 1; }
  grep '^{' gpurun_out/wgp/train_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('  train', d['ms_per_step'], d['value'])"
done
echo done
