#!/bin/bash
# the single-step kernel's prologue stamps (BX_PSTAMPS build in _lib_pst)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pst}; shift
for e in "$@"; do
  BRAX_AMD_LIB=brax_amd/_lib_pst/libbrax_amd.so timeout -k 10 120 python tools/pstamps.py $e > gpurun_out/pstamps_${e}_$TAG.log 2>&1 || exit 2
  grep -v amdgpu.ids gpurun_out/pstamps_${e}_$TAG.log
done
