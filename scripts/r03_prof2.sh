#!/bin/bash
# Round 3: kernel traces of config 3 under the CSR bucket builder (--csr-path bucket: k_bkt_count / place / sort
# per key) and under the bucketed pulls after the batched histogram loads in k_compact.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_oldbkt -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 50 --warmup 2 --no-cpu-baseline --no-buckets --csr-path bucket > gpurun_out/prof_oldbkt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bkt2 -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 50 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bkt2.log 2>&1 || exit 1
for d in prof_oldbkt prof_bkt2; do python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/$d/run_kernel_stats.csv')))
for r in rows[:9]: print('$d', r['Name'][:70], r['Calls'], r['AverageNs'])
"; done
echo done
