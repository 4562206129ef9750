#!/bin/bash
# interleaved A/B of library builds on the bench's Ant loops (1,000 steps, no
# secondary legs): brax_amd/_lib against brax_amd/_lib_<name>, two rounds
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
for round in 1 2; do
  for n in _lib "$@"; do
    lib=brax_amd/$n/libbrax_amd.so; [ "$n" != _lib ] && lib=brax_amd/_lib_$n/libbrax_amd.so
    BRAX_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/abb_${TAG}_${n}_$round.log 2>&1 || { tail -5 gpurun_out/abb_${TAG}_${n}_$round.log; exit 1; }
    echo "$n: $(python tools/bench_line.py gpurun_out/abb_${TAG}_${n}_$round.log)"
  done
done
