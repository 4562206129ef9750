#!/bin/bash
# contact halves: bitwise Ant / Humanoid / HalfCheetah against the base build,
# per-step A/B on HalfCheetah and Pusher, then the HalfCheetah / Pusher / NaN
# parity tests
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06v}
bash tools/gpu_envab.sh $TAG base halfcheetah pusher || exit 3
timeout -k 10 400 python -u -m pytest tests -k "halfcheetah or pusher or cheetah or colliders or capsule" -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -15
