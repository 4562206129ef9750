#!/bin/bash
# interleaved A/B of library builds on one env's kernels (tools/env_ab.py)
set -o pipefail
mkdir -p gpurun_out
TAG=$1; ENV=$2; shift 2
for round in 1 2; do
  for n in _lib "$@"; do
    lib=brax_amd/$n/libbrax_amd.so; [ "$n" != _lib ] && lib=brax_amd/_lib_$n/libbrax_amd.so
    BRAX_AMD_LIB=$lib timeout -k 10 200 python tools/env_ab.py $ENV >> gpurun_out/env_ab_${TAG}_$ENV.log 2>&1 || { tail -5 gpurun_out/env_ab_${TAG}_$ENV.log; exit 1; }
    tail -1 gpurun_out/env_ab_${TAG}_$ENV.log
  done
done
