#!/bin/bash
# round 5: the PK kernels' packed state / AutoReset target through one
# pointer, and the draw-specialised Ant rollout kernel: bitwise rollouts vs
# the previous build, the rollout / graph / env / gym / parity tests, then
# the interleaved A/B on the bench's Ant loops.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05h}
BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -c bitwise gpurun_out/bc_$TAG.log
grep differs gpurun_out/bc_$TAG.log
bash tools/gpu_suite.sh $TAG tests/test_gpu_rollout.py tests/test_gpu_graph.py tests/test_gpu_envs.py tests/test_gpu_gym.py tests/test_gpu_scale.py; [ $? -le 1 ] || exit 5
bash tools/ab_bench.sh $TAG prev || exit 6
bash tools/env_ab.sh $TAG humanoid pd prev || exit 7
bash tools/env_ab.sh $TAG ant prev || exit 8
exit 0
