"""Per-step GPU-vs-golden report for one golden system trajectory (diagnostic).

Prints, per step, the normwise pos/vel error of the HIP path and of the fp32
oracle builds against the float64 golden, and the contact penetrations of
the three where they differ.

  python tests/diag/diag_scene.py box_box
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import brax_amd  # noqa: E402
from brax_amd.base import qp_from_numpy  # noqa: E402
from oracle import oracle as ol  # noqa: E402
from tests.conftest import golden  # noqa: E402
from tests.helpers import compiled, config_for, normwise  # noqa: E402


def main():
  name = sys.argv[1]
  dev = torch.device('cuda', 0)
  sys_ = brax_amd.System(config_for(name), device=dev)
  d, rd = compiled(name)[1:3]
  os32 = [ol.Oracle(d, rd, np.float32, safe_guard=True, fma=f) for f in (False, True)]
  T = golden('traj_' + name)
  np.set_printoptions(precision=6, suppress=True, linewidth=200)
  for t in range(T['action'].shape[0]):
    q, a, ref = T['qp'][t], T['action'][t], T['qp'][t + 1]
    out, info = sys_.step(qp_from_numpy(q, dev), torch.as_tensor(a, dtype=torch.float32,
                                                                 device=dev))
    got = out.numpy()
    pen = info.contact_penetration.cpu().numpy()
    o32 = [o.system_step(q.astype(np.float32), a.astype(np.float32)) for o in os32]
    e = [normwise(got[..., 0:3], ref[..., 0:3]).max(), normwise(got[..., 7:10], ref[..., 7:10]).max()]
    e32 = [max(normwise(x[0][..., 0:3], ref[..., 0:3]).max() for x in o32),
           max(normwise(x[0][..., 7:10], ref[..., 7:10]).max() for x in o32)]
    print(f't={t} gpu pos {e[0]:.2e} vel {e[1]:.2e} | fp32 oracle pos {e32[0]:.2e} vel {e32[1]:.2e}')
    rp = T['contact_penetration'][t]
    if np.abs(pen - rp).max() > 1e-4:
      print('  pen gpu   ', pen.ravel())
      print('  pen golden', rp.ravel())
      print('  pen o32   ', o32[0][1]['contact_penetration'].ravel())
    if e[0] > 1e-4:
      print('  pos gpu   ', got[0, :, 0:3].ravel())
      print('  pos golden', ref[0, :, 0:3].ravel())


if __name__ == '__main__':
  main()
