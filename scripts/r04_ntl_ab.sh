#!/bin/bash
# (The switch was removed from the sources after this measurement; a rebuild of the variant equals the default.)
# Nontemporal LDS-DMA loads in the row kernels (SHPL_ROWS_NTLOAD) against the default library: the conv tests on the
# the variant, then conv and training bench lines with kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=sparse_pooling_amd/variants/libshpl_ntl.so
N=sparse_pooling_amd/libshpl.so
SHPL_LIB=$T timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_grad.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_ntl_tests.log 2>&1 || { tail -30 gpurun_out/r04_ntl_tests.log; exit 1; }
echo "ntl: $(tail -1 gpurun_out/r04_ntl_tests.log)"
bash scripts/ab_args.sh r04_ntlconv "--workload conv --dtype bf16" "k_conv_rows" "base=$N" "ntl=$T" "base2=$N" "ntl2=$T" || exit 1
bash scripts/ab_args.sh r04_ntltrain "--workload conv --train --dtype bf16 --steps 10" "k_conv_rows|k_wgrad_rows<|k_bn_" "base=$N" "ntl=$T" || exit 1
