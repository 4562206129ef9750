#!/bin/bash
# interleaved A/B of the MULTI kernel (tools/multi_ab.py) between
# brax_amd/_lib and brax_amd/_lib_<name> builds: two rounds each
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
for round in 1 2; do
  for n in _lib "$@"; do
    lib=brax_amd/$n/libbrax_amd.so; [ "$n" != _lib ] && lib=brax_amd/_lib_$n/libbrax_amd.so
    BRAX_AMD_LIB=$lib timeout -k 10 200 python tools/multi_ab.py >> gpurun_out/multi_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/multi_ab_$TAG.log; exit 1; }
    tail -1 gpurun_out/multi_ab_$TAG.log
  done
done
