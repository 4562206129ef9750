#!/bin/bash
# MULTI A/B of two library builds (both at their default lanes): bitwise
# states (tools/multi_bitcmp.py), then tools/multi_ab.py interleaved A, B, A,
# B in the early (10 warm steps) and the piled-up (200) state.
#   bash tools/multi_ab_libs.sh <libdir A> <libdir B> <tag>
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
A=${1:-_lib_base}; B=${2:-_lib}; TAG=${3:-ab}
for v in $A $B; do
  BRAX_AMD_LIB=brax_amd/$v/libbrax_amd.so timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_$v.npz > gpurun_out/mbc_$TAG.log 2>&1 || { tail -5 gpurun_out/mbc_$TAG.log; exit 5; }
done
python tools/multi_bitcmp.py cmp gpurun_out/mb_$A.npz gpurun_out/mb_$B.npz | tee gpurun_out/mbcmp_$TAG.log | tail -4
: > gpurun_out/multi_ab_$TAG.log
for warm in 10 200; do
  export BX_MULTI_WARM=$warm
  for rep in 1 2; do
    for v in $A $B; do
      BRAX_AMD_LIB=brax_amd/$v/libbrax_amd.so timeout -k 10 300 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
      tail -1 gpurun_out/mab.tmp | tee -a gpurun_out/multi_ab_$TAG.log
    done
  done
done
