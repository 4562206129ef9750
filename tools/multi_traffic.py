"""Ant Mountain(4) System.step at 2,048 envs with or without the contact-row
Info (diagnostic, for rocprofv3 PMC passes): 30 steps of one mode only, so a
counter pass sees one kind of launch.

    python tools/multi_traffic.py [info|noinfo] [cutoff] [save.npz]

With a third argument the final state is saved (a bitwise A/B of two builds:
BRAX_AMD_LIB selects the library).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import brax_amd  # noqa: E402
from brax_amd.envs.mountain import ant_mountain_config  # noqa: E402


def main():
  info = (sys.argv[1] if len(sys.argv) > 1 else 'noinfo') == 'info'
  cutoff = int(sys.argv[2]) if len(sys.argv) > 2 else 0
  dev = torch.device('cuda', 0)
  cfg = ant_mountain_config(4)
  cfg.collider_cutoff = cutoff
  sys_ = brax_amd.System(cfg, device=dev)
  B = 2048
  qp0 = sys_.default_qp()
  qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                     for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
  act = torch.rand((B, sys_.action_size), device=dev, generator=torch.Generator(dev).manual_seed(0)) * 2 - 1
  qp_bytes = 0
  for _ in range(30):
    qp, inf = sys_.step(qp, act, info=info)
  torch.cuda.synchronize()
  # algorithmic bytes per env-step: the QP in and out (13
  # floats per body), the action row and, with Info, every Info tensor
  qp_bytes = 2 * 13 * 4 * sys_.num_bodies + 4 * sys_.action_size
  info_bytes = 0
  if info:
    def leaves(x):
      if isinstance(x, torch.Tensor):
        yield x
      elif x is not None and hasattr(x, '__dataclass_fields__'):
        for f in x.__dataclass_fields__:
          yield from leaves(getattr(x, f))
    info_bytes = sum(t.numel() * t.element_size() for t in leaves(inf)) // B
  print('mode', 'info' if info else 'noinfo', 'cutoff', cutoff, 'envs', B, 'rows', sys_.num_rows,
        'algorithmic_bytes_per_env_step', qp_bytes + info_bytes, 'info_bytes', info_bytes, flush=True)
  if len(sys.argv) > 3:
    np.savez(sys.argv[3], **{k: getattr(qp, k).cpu().numpy() for k in ('pos', 'rot', 'vel', 'ang')})


if __name__ == '__main__':
  main()
