#!/bin/bash
# Ant env-step throughput vs batch size (waves per SIMD) -> gpurun_out/batch_scan.log
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 4096 8192 16384 32768; do
  timeout -k 10 120 python bench.py --batch $b --steps 300 --warmup 30 --no-cpu-baseline --no-phases --no-secondary > gpurun_out/scan_$b.json 2> gpurun_out/scan_$b.err || { tail -5 gpurun_out/scan_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/scan_$b.json'));print($b, round(d['value']/1e6,2), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4))" | tee -a gpurun_out/batch_scan.log
done
