#!/bin/bash
# rollout output records stored with sc1 (write through, line dropped from the
# XCD's L2: _lib_sc, BX_OUT_SC1) against plain stores: bitwise rollouts, the
# per-launch time over K (tools/diag_rollout_k.py), interleaved
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05ak}
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_base.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
BRAX_AMD_LIB=brax_amd/_lib_sc/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_sc.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_sc.npz gpurun_out/bc_base.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -c bitwise gpurun_out/bc_$TAG.log
for round in 1 2; do
  for lib in _lib _lib_sc; do
    BRAX_AMD_LIB=brax_amd/$lib/libbrax_amd.so timeout -k 10 200 python tools/diag_rollout_k.py 1 20 50 >> gpurun_out/rk_$TAG.log 2>&1 || exit 4
    tail -1 gpurun_out/rk_$TAG.log
  done
done
