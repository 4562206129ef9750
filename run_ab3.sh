#!/bin/bash
# interleaved A/B of library builds on one box (bench only)
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for lib in "$@"; do
  export BRAX_AMD_LIB=$PWD/$lib
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-phases > gpurun_out/bench_ab.log 2>&1 || { tail -3 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$lib', round(d['value']/1e6,2),'M/s kernel_ms',round(d['roofline']['kernel_ms'],4),'ms/step',round(d['ms_per_step'],4))"
done
done
