#!/bin/bash
# A/B of library builds (brax_amd/_lib and the brax_amd/_lib_<name> given):
# the bench's Ant loops at 1,000 steps, then HalfCheetah / Humanoid kernels
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
for n in _lib "$@"; do
  lib=brax_amd/$n/libbrax_amd.so; [ "$n" != _lib ] && lib=brax_amd/_lib_$n/libbrax_amd.so
  BRAX_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/ablib_${TAG}_$n.log 2>&1 || { tail -5 gpurun_out/ablib_${TAG}_$n.log; exit 1; }
  echo "$n: $(python tools/bench_line.py gpurun_out/ablib_${TAG}_$n.log)"
  for e in halfcheetah humanoid; do
    BRAX_AMD_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ablib_${TAG}_${n}_$e -o run --output-format csv -- python3 tools/env_prof.py $e > gpurun_out/ablib_${TAG}_${n}_$e.log 2>&1 || { tail -5 gpurun_out/ablib_${TAG}_${n}_$e.log; exit 1; }
    python3 - gpurun_out/ablib_${TAG}_${n}_$e <<'PY'
import csv, sys
v = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in csv.DictReader(open(sys.argv[1] + '/run_kernel_trace.csv')) if 'env_step' in r['Kernel_Name']]
print('  ', sys.argv[1].split('_')[-1], round(sum(v) / len(v) / 1e3, 2), 'us')
PY
  done
done
