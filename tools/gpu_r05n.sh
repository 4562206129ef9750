#!/bin/bash
# MULTI-mode phase stamps (BX_MSTAMPS build, broad phase split out), then the
# MULTI variants: default (256 lanes, 2 waves/SIMD), BX_MULTI_RELOAD (joint,
# gather lists and tasks re-read per phase) at 2 and 3 waves/SIMD, and 128
# lanes per env (BX_MULTI_L=128): bitwise states against the default, the
# MULTI parity tests under each, then the interleaved timing A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05n}
for cut in 0 36; do
  BRAX_AMD_LIB=brax_amd/_lib_mst/libbrax_amd.so timeout -k 10 200 python tools/mstamps.py $cut > gpurun_out/mstamps_${TAG}_$cut.log 2>&1 || exit 3
  grep -v amdgpu.ids gpurun_out/mstamps_${TAG}_$cut.log
done
timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_base.npz > gpurun_out/mbc_$TAG.log 2>&1 || exit 5
for v in "_lib_rl 2 256" "_lib_rl 3 256" "_lib 2 128" "_lib_rl 2 128"; do
  set -- $v
  BX_MULTI_WPE=$2 BX_MULTI_L=$3 BRAX_AMD_LIB=brax_amd/$1/libbrax_amd.so timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_v.npz >> gpurun_out/mbc_$TAG.log 2>&1 || exit 5
  echo "== $v" | tee -a gpurun_out/mbc_$TAG.log
  python tools/multi_bitcmp.py cmp gpurun_out/mb_base.npz gpurun_out/mb_v.npz | tee -a gpurun_out/mbc_$TAG.log | grep -c bitwise
done
for v in "_lib_rl 3 256" "_lib 2 128"; do
  set -- $v
  BX_MULTI_WPE=$2 BX_MULTI_L=$3 BRAX_AMD_LIB=brax_amd/$1/libbrax_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mountain" > gpurun_out/pyt_mv_$TAG.log 2>&1 || { tail -20 gpurun_out/pyt_mv_$TAG.log; exit 6; }
  echo "== $v $(tail -1 gpurun_out/pyt_mv_$TAG.log)"
done
for round in 1 2; do
  for v in "_lib 2 256" "_lib_rl 2 256" "_lib_rl 3 256" "_lib 2 128" "_lib_rl 2 128"; do
    set -- $v
    BX_MULTI_WPE=$2 BX_MULTI_L=$3 BRAX_AMD_LIB=brax_amd/$1/libbrax_amd.so timeout -k 10 200 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
    echo "wpe=$2 L=$3 $(tail -1 gpurun_out/mab.tmp)" | tee -a gpurun_out/multi_ab_$TAG.log
  done
done
