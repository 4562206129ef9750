#!/bin/bash
# GPU session helper: tests -> smoke -> short bench; stops on the first failure.
# usage: bash tools/run_gpu.sh [tag] [extra bench args]
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
shift
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python - <<PY
import json
d = json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1])
r = d['roofline']
print('value', round(d['value'] / 1e6, 2), 'M/s; ms/step', round(d['ms_per_step'], 4),
      '; kernel_ms', round(r['kernel_ms'], 4), '; valu frac', round(r['frac'], 4))
print(json.dumps(d.get('secondary_configs')))
PY
exit $rc
