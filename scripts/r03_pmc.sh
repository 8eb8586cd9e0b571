#!/bin/bash
# PMC HBM traffic (FETCH_SIZE and WRITE_SIZE: one pass each, separate runs) of every bench workload the
# bench line looks up in profiles/traffic.json, on the library in this tree: gpurun_out/pmc_<tag>_<counter>/
# and the profiled bench's own line (its lib_sha256) in gpurun_out/pmc_<tag>_<counter>.log. Then locally:
#   python scripts/traffic.py step <key> <tag> [all] [anchor]   (stamps the entry with that lib_sha256; anchor:
#   the kernel launched once per step -- k_count, or k_bev_frame for the raw-scan step, whose velodyne
#   stage launches k_count too)
# WHICH: space-separated subset of the tags below (default: all).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
declare -A ARGS=(
  [c2f64]="--config 2 --no-pool-report"
  [c2f8]="--config 2 --frames 8 --no-pool-report"
  [c3f4]="--config 3"
  [c5f64]="--config 5"
  [frf64]="--workload frames"
  [frbev]="--workload frames --maps-form bev_input"
  [trbf16]="--workload conv --train --dtype bf16"
)
for tag in ${WHICH:-c2f64 c2f8 c3f4 c5f64 frf64 frbev trbf16}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "shpl" \
      -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- \
      python3 bench.py ${ARGS[$tag]} --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_${tag}_$c.log 2>&1
    rc=$?; echo "pmc $tag $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_${tag}_$c.log; exit $rc; }
  done
done
if [ -n "$CONV" ]; then  # the conv workloads' per-call traffic (traffic.py conv_<dt>_F64)
  for dt in $CONV; do DT=$dt bash scripts/gpu_conv_prof.sh || exit 1; done
fi
echo done
