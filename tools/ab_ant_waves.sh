#!/bin/bash
# A/B of the Ant step kernel's register cap: this tree's library against
# brax_amd/_lib_w1 (built with -DBX_ANT_WAVES=1), 4,096 and 32,768 envs
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-ab}
for lib in brax_amd/_lib/libbrax_amd.so brax_amd/_lib_w1/libbrax_amd.so; do
  n=$(basename $(dirname $lib))
  BRAX_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-phases --no-cpu-baseline > gpurun_out/ab_${TAG}_$n.log 2>&1 || { tail -5 gpurun_out/ab_${TAG}_$n.log; exit 1; }
  echo $n; grep '^{' gpurun_out/ab_${TAG}_$n.log | python -c "
import json,sys
d=json.loads(sys.stdin.read().splitlines()[-1]); s=d['secondary_configs']
print(' single-step kernel us', round(d['roofline']['single_step_kernel_ms']*1e3,2), 'value M', round(d['value']/1e6,1), 'ant32768 M', round(s['ant_32768_one_gpu']['value']/1e6,1), 'humanoid M', round(s['humanoid_4096']['value']/1e6,1))"
done
