#!/bin/bash
# A/B of the step kernel's threads per workgroup (64 vs 32) -> gpurun_out/ab_block.log
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 64 32 64 32; do
  timeout -k 10 300 python bench.py --block $b --no-cpu-baseline --no-phases --no-secondary > gpurun_out/ab_$b.json 2> gpurun_out/ab_$b.err || { tail -5 gpurun_out/ab_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$b.json'));print('block $b', round(d['value']/1e6,2), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4))" | tee -a gpurun_out/ab_block.log
done
