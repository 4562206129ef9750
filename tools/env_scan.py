"""Env.step rate of every registered env at 4,096 envs on one GPU: a fixed
U[-1,1] action slab, episode_length 1000 with auto-reset, 100 timed steps
after 10 warm ones (HIP events), plus the step kernel's instantiation.

    python tools/env_scan.py [--batch 4096] [--steps 100]
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

ENVS = ['ant', 'humanoid', 'humanoidstandup', 'halfcheetah', 'hopper', 'walker2d', 'swimmer',
        'reacher', 'reacherangle', 'pusher', 'ur5e', 'fetch', 'grasp', 'inverted_pendulum',
        'inverted_double_pendulum', 'acrobot']


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--batch', type=int, default=4096)
  ap.add_argument('--steps', type=int, default=100)
  args = ap.parse_args()
  warnings.filterwarnings('ignore')
  from brax_amd import envs
  dev = torch.device('cuda', 0)
  B = args.batch
  out = {}
  for name in ENVS:
    env = envs.create(name, batch_size=B, episode_length=1000, auto_reset=True, device=dev)
    st = env.reset(np.array([0, 1], np.uint32))
    act = torch.rand((B, env.action_size), device=dev) * 2 - 1
    for _ in range(10):
      st = env.step(st, act)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for _ in range(args.steps):
      st = env.step(st, act)
    b.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    u = env.unwrapped
    out[name] = {'env_steps_per_s': B * args.steps / wall,
                 'gpu_us_per_step': a.elapsed_time(b) * 1e3 / args.steps,
                 'bodies': u.sys.num_bodies, 'obs': u.obs_size, 'actions': env.action_size,
                 'lanes_per_env': getattr(u.sys, 'lanes', None)}
    print(name, json.dumps(out[name]), flush=True)
    del env, st, act
  print(json.dumps({'batch': B, 'steps': args.steps, 'envs': out}), flush=True)


if __name__ == '__main__':
  main()
