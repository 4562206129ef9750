#!/bin/bash
# the bench's N-rank path on ONE GPU: `python bench.py --gpus 2` (the parent
# spawns the two ranks itself, as the driver's `--gpus N` run does), gloo
# collectives (RCCL refuses two ranks on one device), both ranks on cuda:0.
# Checks the rank sharding, barrier + max-over-ranks timing, the episodic
# exchange inside the timed region (collectives_in_timed_region) and rank 0's
# line with n_gpus 2. MODE=torchrun: the same under torchrun.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r}; STEPS=${2:-20}; WARM=${3:-5}
if [ "$MODE" = torchrun ]; then
  BX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps $STEPS --warmup $WARM \
    --no-phases --no-secondary > gpurun_out/bench_2rank_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_2rank_$TAG.log; exit 1; }
else
  BX_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps $STEPS --warmup $WARM \
    --no-phases --no-secondary > gpurun_out/bench_2rank_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_2rank_$TAG.log; exit 1; }
fi
grep '^{' gpurun_out/bench_2rank_$TAG.log | python -c "
import json, sys
d = json.loads(sys.stdin.read().splitlines()[-1])
assert d['n_gpus'] == 2, d['n_gpus']
print('n_gpus', d['n_gpus'], 'parallelism', d['config']['parallelism'], 'timed', d['timed_loop'],
      'collectives_in_timed_region', d['collectives_in_timed_region'],
      {k: d[k].get('collectives_in_timed_region') for k in ('eager_loop', 'graph_loop', 'rollout_loop', 'direct_loop') if k in d})"
