#!/bin/bash
# SINGLE env rollouts bitwise against _lib_prev (r05g), Humanoid A/B, the GPU suite
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05ab}
BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -v amdgpu.ids gpurun_out/bc_$TAG.log | grep -v bitwise; grep -c bitwise gpurun_out/bc_$TAG.log
bash tools/env_ab.sh $TAG humanoid prev || exit 4
bash tools/gpu_suite.sh $TAG
