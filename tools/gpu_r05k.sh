#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for n in _lib _lib_prev; do
  BRAX_AMD_LIB=brax_amd/$n/libbrax_amd.so timeout -k 10 200 python tools/diag_rollout_k.py 2>&1 | grep -v amdgpu.ids || exit 2
done
