"""A/B of the spherical joint halves (diagnostic): Humanoid at 4,096 envs,
the 32-lane env kernels (default) against the 16-lane kernel
(BX_SPH_HALVES=0), HIP events over back-to-back Env.step calls of one fixed
action slab and over 50-step rollout launches.

    python tools/sph_ab.py [envs]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import envs  # noqa: E402
from brax_amd.envs.rollout import rollout  # noqa: E402


def timed(fn, n):
  for _ in range(3):
    fn()
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  a.record()
  for _ in range(n):
    fn()
  b.record()
  torch.cuda.synchronize()
  return a.elapsed_time(b) * 1e3 / n


def main():
  B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
  dev = torch.device('cuda', 0)
  res = {}
  for halves in (False, True, False, True):
    os.environ['BX_SPH_HALVES'] = '1' if halves else '0'
    env = envs.create('humanoid', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
    st = [env.reset(np.array([0, 3], np.uint32))]
    g = torch.Generator(dev).manual_seed(1)
    act = torch.rand((B, env.action_size), device=dev, generator=g) * 2 - 1
    acts = torch.rand((50, B, env.action_size), device=dev, generator=g) * 2 - 1

    def step():
      st[0] = env.step(st[0], act)

    def roll():
      st[0] = rollout(env, st[0], acts)[0]
    us_step = timed(step, 50)
    us_roll = timed(roll, 4) / 50
    lanes = env.unwrapped.sys.env_lanes
    res.setdefault(lanes, []).append((us_step, us_roll))
    print(f'humanoid B={B} env lanes {lanes}: Env.step {us_step:.2f} us, rollout {us_roll:.2f} us/step',
          flush=True)
  for lanes, v in sorted(res.items()):
    print(f'lanes {lanes}: best Env.step {min(x[0] for x in v):.2f} us, best rollout '
          f'{min(x[1] for x in v):.2f} us/step', flush=True)


if __name__ == '__main__':
  main()
