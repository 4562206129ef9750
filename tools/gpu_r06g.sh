#!/bin/bash
# MULTI-mode phase stamps of the compact-contacts build (BX_MSTAMPS,
# brax_amd/_lib_mst), cutoff 0 and 36
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06g}
for cut in 0 36; do
  BRAX_AMD_LIB=brax_amd/_lib_mst/libbrax_amd.so timeout -k 10 200 python tools/mstamps.py $cut > gpurun_out/mstamps_${TAG}_$cut.log 2>&1 || exit 3
  grep -v amdgpu.ids gpurun_out/mstamps_${TAG}_$cut.log
done
