#!/bin/bash
# The full GPU record of one build: GPU tests, smoke, default bench (with the
# CPU baseline), rocprof + PMC passes, per-env kernel profiles, the driver's
# 20-step command twice + a 1,000-step bench, the rollout K sweep.
#   bash tools/gpu_round.sh TAG
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r}
bash tools/gpu_tests.sh $TAG || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash tools/run_bench.sh $TAG || exit 1
bash tools/run_prof.sh $TAG || exit 1
bash tools/run_env_prof.sh $TAG ant humanoid humanoidstandup halfcheetah pusher fetch hopper walker2d || exit 1
bash tools/gpu_quick.sh $TAG || exit 1
timeout -k 10 200 python tools/rollout_k.py 10 20 50 > gpurun_out/rollout_k_$TAG.log 2>&1 || exit 1
tail -n 4 gpurun_out/rollout_k_$TAG.log
