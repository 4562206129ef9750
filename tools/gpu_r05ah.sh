#!/bin/bash
# lane image loaded by the wave's first env and broadcast (BX_IMG_BCAST,
# _lib_bc) against the default: bitwise rollouts, Ant / Humanoid A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05ah}
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_base.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
BRAX_AMD_LIB=brax_amd/_lib_bc/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_bc.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_base.npz gpurun_out/bc_bc.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -c bitwise gpurun_out/bc_$TAG.log
for e in ant humanoid; do bash tools/env_ab.sh $TAG $e bc || exit 4; done
