#!/bin/bash
# A/B of brax_amd/_lib_<x> builds against _lib: bitwise Ant / Humanoid /
# HalfCheetah rollouts, per-step times of the envs named
#   bash tools/gpu_libab.sh <tag> <x> env...
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; X=$2; shift 2
for v in _lib _lib_$X; do
  BRAX_AMD_LIB=brax_amd/$v/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc$v.npz > gpurun_out/bc_$TAG.log 2>&1 || { tail -5 gpurun_out/bc_$TAG.log; exit 5; }
done
python tools/bitcmp.py cmp gpurun_out/bc_lib.npz gpurun_out/bc_lib_$X.npz > gpurun_out/bitcmp_$TAG.log
grep -c bitwise gpurun_out/bitcmp_$TAG.log; grep differs gpurun_out/bitcmp_$TAG.log
for e in "$@"; do
  bash tools/env_ab.sh $TAG $e $X || exit 6
done
