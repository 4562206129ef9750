#!/bin/bash
# round 6 first look: the NaN / Inf goldens on the HIP path (all failures
# listed), then the Mountain tests after the MULTI staging barrier
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06a}
timeout -k 10 400 python -u -m pytest tests/test_gpu_nan.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_nan_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_nan_$TAG.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mountain" -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mtn_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_mtn_$TAG.log; exit 6; }
tail -2 gpurun_out/pytest_mtn_$TAG.log
