#!/bin/bash
# Per-step PMC HBM traffic of the bf16 training step and the raw-scan step (every SHPL kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=trainbf16 KREGEX=shpl BENCH_ARGS="--workload conv --train --dtype bf16" bash scripts/r02_pmc.sh || exit 1
TAG=frames KREGEX=shpl BENCH_ARGS="--workload frames" bash scripts/r02_pmc.sh || exit 1
echo done
