#!/bin/bash
# NaN-faithful masks / flags on the default build: the NaN, EvalWrapper and
# MULTI-vs-item-loop tests, then the cost against HEAD's library
# (brax_amd/_lib_prev), interleaved
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06c}
timeout -k 10 500 python -u -m pytest tests/test_gpu_nan.py tests/test_gpu_eval.py "tests/test_gpu_scale.py::test_mountain4_multi_vs_item_loops" -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_new_$TAG.log 2>&1
rc=$?
cp gpurun_out/parity_margins.json gpurun_out/margins_new_$TAG.json 2>/dev/null
grep -E "PASSED|FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_new_$TAG.log | tail -20
[ $rc -le 1 ] || exit $rc
bash tools/env_ab.sh $TAG ant prev || exit 3
bash tools/env_ab.sh $TAG humanoid prev || exit 3
for n in _lib _lib_prev _lib _lib_prev; do
  BRAX_AMD_LIB=brax_amd/$n/libbrax_amd.so timeout -k 10 200 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
  tail -1 gpurun_out/mab.tmp | tee -a gpurun_out/multi_ab_$TAG.log
done
