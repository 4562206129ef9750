#!/bin/bash
# SLP-vectorised fast TU (_lib_slp) against _lib: bitwise rollouts, then the
# interleaved per-env A/B on the three hot envs
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05m}
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_base.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
BRAX_AMD_LIB=brax_amd/_lib_slp/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_slp.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_base.npz gpurun_out/bc_slp.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -v amdgpu.ids gpurun_out/bc_$TAG.log | tail -18
for e in ant humanoid halfcheetah; do bash tools/env_ab.sh $TAG $e slp || exit 4; done
