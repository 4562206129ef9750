#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in "$@"; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-cpu-baseline --variant $v > gpurun_out/bench_var.log 2>&1 || { tail -5 gpurun_out/bench_var.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_var.log').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,2),'M/s kernel_ms',round(d['roofline']['kernel_ms'],4),'ms/step',round(d['ms_per_step'],4))"
done
done
