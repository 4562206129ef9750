#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu.log | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "" "--generic" "" "--generic"; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-cpu-baseline $v > gpurun_out/bench_ab.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,2),'M/s kernel_ms',round(d['roofline']['kernel_ms'],4),'ms/step',round(d['ms_per_step'],4))"
done
