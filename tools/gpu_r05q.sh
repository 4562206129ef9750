#!/bin/bash
# MULTI roles rotated by workgroup (BX_MULTI_ROT: body / joint lanes on wave
# blockIdx % 4) against the default: bitwise states, the A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05q}
timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_base.npz > gpurun_out/mbc_$TAG.log 2>&1 || exit 5
BRAX_AMD_LIB=brax_amd/_lib_rot/libbrax_amd.so timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_new.npz >> gpurun_out/mbc_$TAG.log 2>&1 || exit 5
python tools/multi_bitcmp.py cmp gpurun_out/mb_base.npz gpurun_out/mb_new.npz | tee -a gpurun_out/mbc_$TAG.log
bash tools/multi_ab.sh $TAG rot
