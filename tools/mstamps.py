"""Diagnostic: per-phase cycle shares of the MULTI-mode step (BX_MSTAMPS build),
Ant Mountain(4), 2048 envs; argv[1] = NearNeighbors cutoff (default 0)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import brax_amd  # noqa: E402
from brax_amd import _native  # noqa: E402
from brax_amd.envs.mountain import ant_mountain_config  # noqa: E402

cut = int(sys.argv[1]) if len(sys.argv) > 1 else 0
dev = torch.device('cuda', 0)
cfg = ant_mountain_config(4)
cfg.collider_cutoff = cut
sys_ = brax_amd.System(cfg, device=dev)
B = 2048
qp0 = sys_.default_qp()
qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                   for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
lib = _native.lib()
buf = (C.c_ulonglong * 16)()
for k in range(30):
  if k == 5:
    torch.cuda.synchronize()
    _native.check(lib.bx_debug_stamps(buf, 3))
  a = torch.rand((B, sys_.action_size), device=dev) * 2 - 1
  qp, _ = sys_.step(qp, a)
torch.cuda.synchronize()
_native.check(lib.bx_debug_stamps(buf, 2))
v = np.array(buf[:12], dtype=np.float64)
n = max(buf[15], 1)
names = ['act+damp', 'body acc', 'joint', 'body pos(+vproj)', 'contacts + listing',
         'pos impulses + tasks', 'body combine pos', 'vel impulses + tasks', 'body combine vel',
         'nn select', 'tail', 'broad phase']
if cut:
  # (culled scenes: slots 12-14 split the NearNeighbors picks)
  print('nn: init loop', buf[14] / n, 'keys + sort', buf[12] / n, 'wave picks', buf[13] / n,
        'merge (rest of nn select)', buf[9] / n)
else:
  print('near rows per broad-phase pass', buf[12] / max(buf[13], 1), 'passes/wg-step', buf[13] / n,
        'listed (penetrating) rows per pass', buf[14] / (n * (sys_.config.substeps // 2)))
tot = v.sum()
print('cutoff', cut, 'samples', n, 'cycles/wave0/step', tot / n)
for i, nm in enumerate(names):
  print(f'{nm:24s} {100 * v[i] / tot:5.1f}%  {v[i] / n:9.0f} cyc')
