#!/bin/bash
# Humanoid: the observation's centre of mass reused as the next step's
# (default) against recomputing it (_lib_nc, BX_NO_COM_KEEP): bitwise
# rollouts, the rollout / env tests, the Humanoid A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05aj}
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_base.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
BRAX_AMD_LIB=brax_amd/_lib_nc/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_nc.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_nc.npz gpurun_out/bc_base.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -c bitwise gpurun_out/bc_$TAG.log
grep -v bitwise gpurun_out/bc_$TAG.log | grep -v amdgpu.ids | tail -8
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_envs.py tests/test_gpu_gym.py > gpurun_out/pyt_h_$TAG.log 2>&1 || { tail -30 gpurun_out/pyt_h_$TAG.log; exit 6; }
tail -1 gpurun_out/pyt_h_$TAG.log
bash tools/env_ab.sh $TAG humanoid nc
