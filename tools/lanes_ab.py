"""A/B of lanes per env (diagnostic): an env's step at 4,096 envs on its
default kernel, then with the system set to 32 lanes per env
(`bx_system_set_variant(32, SINGLE)`: two envs per wave, two waves per SIMD,
the all-kinds SINGLE kernel), HIP events over 50 back-to-back Env.step calls
of one fixed action slab.

    python tools/lanes_ab.py humanoid ant
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import _native, envs  # noqa: E402


def step_us(env, st, act, n=50):
  for _ in range(5):
    st = env.step(st, act)
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  a.record()
  for _ in range(n):
    st = env.step(st, act)
  b.record()
  torch.cuda.synchronize()
  return a.elapsed_time(b) * 1e3 / n


def main():
  dev = torch.device('cuda', 0)
  for name in sys.argv[1:] or ['humanoid']:
    env = envs.create(name, batch_size=4096, episode_length=1000, auto_reset=True, device=dev)
    st = env.reset(np.array([0, 3], np.uint32))
    act = torch.rand((4096, env.action_size), device=dev, generator=torch.Generator(dev).manual_seed(1)) * 2 - 1
    base = step_us(env, st, act)
    u = env.unwrapped
    rc = _native.lib().bx_system_set_variant(u.sys._h, 32, 1)
    if rc != 0:
      print(name, 'default', round(base, 2), 'us; 32 lanes refused:', _native.lib().bx_last_error().decode())
      continue
    wide = step_us(env, st, act)
    print(f'{name}: default kernel {base:.2f} us/step, 32 lanes per env {wide:.2f} us/step '
          f'({base / wide:.3f}x)', flush=True)


if __name__ == '__main__':
  main()
