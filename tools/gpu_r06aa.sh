#!/bin/bash
# Pusher-specialised env kernels: per-step A/B against the base build and the
# Pusher tests
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06aa}
bash tools/gpu_envab.sh $TAG base pusher || exit 3
timeout -k 10 400 python -u -m pytest tests -k "pusher" -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -8
