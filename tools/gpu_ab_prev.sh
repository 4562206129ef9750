# a kernel-source change against the previous build (brax_amd/_lib_prev): the
# bitwise comparison of 20-step Ant / Humanoid / HalfCheetah rollouts, then
# the A/B bench (tools/ab_libs.sh)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-ab}
BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
bash tools/ab_libs.sh $TAG prev
