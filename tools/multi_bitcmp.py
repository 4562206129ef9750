"""Diagnostic: Ant Mountain(4) System.step states (2,048 envs, 10 steps,
cutoff 0 and 36, Info on) on the library / knobs of this process, saved for a
bitwise comparison between MULTI-kernel variants.

  BRAX_AMD_LIB=<lib> [BX_MULTI_LANES=128|256] python tools/multi_bitcmp.py save <out.npz>
  python tools/multi_bitcmp.py cmp <a.npz> <b.npz>
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(path):
  import torch
  import brax_amd
  from brax_amd.envs.mountain import ant_mountain_config
  dev = torch.device('cuda', 0)
  B = 2048
  out = {}
  for cut in (0, 36):
    cfg = ant_mountain_config(4)
    cfg.collider_cutoff = cut
    s = brax_amd.System(cfg, device=dev)
    if os.environ.get('BX_MULTI_LANES'):
      from brax_amd import _native
      _native.check(_native.lib().bx_system_set_variant(s._h, int(os.environ['BX_MULTI_LANES']), 3))
    qp0 = s.default_qp()
    qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                       for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
    g = torch.Generator(device=dev).manual_seed(11 + cut)
    info = None
    for _ in range(10):
      a = torch.rand((B, s.action_size), device=dev, generator=g) * 2 - 1
      qp, info = s.step(qp, a)
    torch.cuda.synchronize()
    for f in ('pos', 'rot', 'vel', 'ang'):
      out[f'c{cut}_{f}'] = getattr(qp, f).cpu().numpy()
    out[f'c{cut}_pen'] = info.contact_penetration.cpu().numpy()
    # Info off: the broad phase on the last pass too
    q2 = qp
    for _ in range(3):
      a = torch.rand((B, s.action_size), device=dev, generator=g) * 2 - 1
      q2, _ = s.step(q2, a, info=False)
    torch.cuda.synchronize()
    for f in ('pos', 'vel'):
      out[f'c{cut}_noinfo_{f}'] = getattr(q2, f).cpu().numpy()
  np.savez(path, **out)


def cmp(a, b):
  A, Bz = np.load(a), np.load(b)
  for k in A.files:
    x, y = A[k], Bz[k]
    if np.array_equal(x.view(np.uint32), y.view(np.uint32)):
      print(k, 'bitwise')
    else:
      print(k, 'DIFF max', float(np.nanmax(np.abs(x - y))))


if __name__ == '__main__':
  {'save': save, 'cmp': cmp}[sys.argv[1]](*sys.argv[2:])
