# the default build and the no-phase-barrier build (brax_amd/_lib_nosync)
# against the previous build (brax_amd/_lib_prev): bitwise 20-step rollouts,
# then the A/B bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-abn}
BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
BRAX_AMD_LIB=brax_amd/_lib_nosync/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_nosync.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
echo "== default vs prev" >> gpurun_out/bc_$TAG.log
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
echo "== nosync vs prev" >> gpurun_out/bc_$TAG.log
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_nosync.npz >> gpurun_out/bc_$TAG.log 2>&1
bash tools/ab_libs.sh $TAG prev nosync
