#!/bin/bash
# the build without -fno-honor-nans / -fno-honor-infinities (FINITE=0,
# brax_amd/_lib_hn): the NaN goldens on it, then its cost (interleaved A/B
# against brax_amd/_lib: Ant / Humanoid rollout and Env.step, Mountain(4))
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06b}
BRAX_AMD_LIB=brax_amd/_lib_hn/libbrax_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_nan.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_nan_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_nan_$TAG.log | tail -14
[ $rc -le 1 ] || exit $rc
bash tools/env_ab.sh $TAG ant hn || exit 3
bash tools/env_ab.sh $TAG humanoid hn || exit 3
for n in _lib _lib_hn; do
  BRAX_AMD_LIB=brax_amd/$n/libbrax_amd.so timeout -k 10 200 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
  tail -1 gpurun_out/mab.tmp | tee -a gpurun_out/multi_ab_$TAG.log
done
