set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --workload conv --no-cpu-baseline > gpurun_out/cf.log 2>&1 && \
timeout -k 10 200 python bench.py --workload conv --train --no-cpu-baseline > gpurun_out/cft.log 2>&1 && \
timeout -k 10 200 python bench.py --workload conv --train --dtype bf16 --no-cpu-baseline > gpurun_out/cbt.log 2>&1
rc=$?
for f in cf cft cbt; do python3 -c "
import json,sys
for l in open('gpurun_out/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('kernel_ms'), d.get('unfused'))"; done
exit $rc
