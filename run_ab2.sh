#!/bin/bash
# A/B two library builds: parity tests + bench for each.
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in "$@"; do
  export BRAX_AMD_LIB=$PWD/$lib
  timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1
  rc=$?
  echo "== $lib pytest rc=$rc"; grep -E "passed|failed|normwise" gpurun_out/pytest_ab.log | tail -8
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for rep in 1 2; do
for lib in "$@"; do
  export BRAX_AMD_LIB=$PWD/$lib
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-cpu-baseline --no-phases > gpurun_out/bench_ab.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$lib', round(d['value']/1e6,2),'M/s kernel_ms',round(d['roofline']['kernel_ms'],4),'ms/step',round(d['ms_per_step'],4))"
done
done
