#!/bin/bash
# A/B of library builds (BRAX_AMD_LIB) on the bench lines -> gpurun_out/ab_lib.log
# usage: bash run_ab_lib.sh <dir> [<dir> ...]   (dirs under brax_amd/, "_lib" = default)
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for d in "$@"; do
    export BRAX_AMD_LIB=$PWD/brax_amd/$d/libbrax_amd.so
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-phases > gpurun_out/ab_$d.json 2> gpurun_out/ab_$d.err || { tail -5 gpurun_out/ab_$d.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$d.json'));print('$d', round(d['value']/1e6,2), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'humanoid', round(d['secondary_configs']['humanoid_4096']['value']/1e6,2), 'mountain', round(d['secondary_configs']['mountain4_2048_cutoff0']['value']/1e6,3))" | tee -a gpurun_out/ab_lib.log
  done
done
