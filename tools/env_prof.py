"""One env's Env.step at 4,096 envs for rocprofv3 passes (kernel trace, SQ
counters): 5 warm + 20 steps of one fixed action slab, then the step rate.

    python tools/env_prof.py pusher [--batch 4096] [--steps 20]
"""
import argparse
import json
import os
import sys
import time
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('name')
  ap.add_argument('--batch', type=int, default=4096)
  ap.add_argument('--steps', type=int, default=20)
  ap.add_argument('--block', type=int, default=0, help='threads per workgroup (A/B)')
  args = ap.parse_args()
  warnings.filterwarnings('ignore')
  from brax_amd import envs
  dev = torch.device('cuda', 0)
  B = args.batch
  env = envs.create(args.name, batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  if args.block:
    from brax_amd import _native
    _native.check(_native.lib().bx_system_set_block(env.unwrapped.sys._h, args.block))
  st = env.reset(np.array([0, 1], np.uint32))
  act = torch.rand((B, env.action_size), device=dev) * 2 - 1
  for _ in range(5):
    st = env.step(st, act)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    st = env.step(st, act)
  torch.cuda.synchronize()
  wall = time.perf_counter() - t0
  print(json.dumps({'env': args.name, 'env_steps_per_s': B * args.steps / wall,
                    'us_per_step': wall * 1e6 / args.steps,
                    'lanes_per_env': env.unwrapped.sys.lanes}), flush=True)


if __name__ == '__main__':
  main()
