"""Diagnostic: Ant rollout kernel time per launch for K steps, actions given
(bx_env_rollout_packed) vs drawn in the launch (RolloutRunner), on the
library BRAX_AMD_LIB names."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, n=10):
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
  from brax_amd import envs
  from brax_amd.envs.rollout import RolloutRunner, rollout
  dev = torch.device('cuda', 0)
  env = envs.create('ant', batch_size=4096, episode_length=1000, auto_reset=True, device=dev)
  st = env.reset(np.array([0, 7], np.uint32))
  out = {}
  ks = [int(k) for k in sys.argv[1:]] or [1, 5, 20]
  for K in ks:
    acts = torch.rand((K, 4096, 8), device=dev) * 2 - 1
    buf = torch.empty((K * 4096 * (160 + 87 + 4 + 10),), device=dev)
    out[f'given K={K}'] = timed(lambda: rollout(env, st, acts, out=buf)) / K
    r = RolloutRunner(env, st, K, seed=3)
    out[f'drawn K={K}'] = timed(r.run) / K
    out[f'drawn K={K} launch'] = out[f'drawn K={K}'] * K
  print(os.environ.get('BRAX_AMD_LIB', '_lib'), {k: round(v, 2) for k, v in out.items()}, flush=True)


if __name__ == '__main__':
  main()
