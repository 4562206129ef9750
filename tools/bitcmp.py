"""Diagnostic: one library build's Ant / Humanoid / HalfCheetah rollouts (4096 envs, 20
steps, fixed seeds) saved for a bitwise comparison between builds.

  BRAX_AMD_LIB=<lib> python tools/bitcmp.py save <out.npz>
  python tools/bitcmp.py cmp <a.npz> <b.npz>
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(path):
  import torch
  from brax_amd import envs
  dev = torch.device('cuda', 0)
  out = {}
  for name in ('ant', 'humanoid', 'halfcheetah'):
    env = envs.create(name, batch_size=4096, episode_length=1000, auto_reset=True, device=dev)
    st = env.reset(np.array([0, 7], np.uint32))
    g = torch.Generator(dev).manual_seed(3)
    for _ in range(20):
      st = env.step(st, torch.rand((4096, env.action_size), device=dev, generator=g) * 2 - 1)
    torch.cuda.synchronize()
    for f in ('pos', 'rot', 'vel', 'ang'):
      out[f'{name}_{f}'] = getattr(st.qp, f).cpu().numpy()
    out[f'{name}_obs'] = st.obs.cpu().numpy()
    out[f'{name}_reward'] = st.reward.cpu().numpy()
  np.savez(path, **out)


def cmp(a, b):
  x, y = np.load(a), np.load(b)
  bad = [k for k in x.files if not np.array_equal(x[k].view(np.uint32), y[k].view(np.uint32))]
  for k in x.files:
    d = np.abs(x[k].astype(np.float64) - y[k]).max()
    print(k, 'bitwise' if k not in bad else f'differs (max {d:.3g})')
  return 1 if bad else 0


if __name__ == '__main__':
  if sys.argv[1] == 'save':
    save(sys.argv[2])
  else:
    sys.exit(cmp(sys.argv[2], sys.argv[3]))
