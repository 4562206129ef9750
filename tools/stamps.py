"""Diagnostic: per-phase cycle shares of the single-mode step (BX_STAMPS build)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import _native, envs  # noqa: E402

dev = torch.device('cuda', 0)
name = sys.argv[1] if len(sys.argv) > 1 else 'ant'
env = envs.create(name, batch_size=4096, episode_length=1000, device=dev)
st = env.reset(np.array([0, 1], np.uint32))
lib = _native.lib()
buf = (C.c_ulonglong * 16)()
for k in range(60):
  if k == 10:
    torch.cuda.synchronize()
    _native.check(lib.bx_debug_stamps(buf, 1))
  a = torch.rand((4096, env.action_size), device=dev) * 2 - 1
  st = env.step(st, a)
torch.cuda.synchronize()
_native.check(lib.bx_debug_stamps(buf, 0))
v = np.array(buf[:10], dtype=np.float64)
n = buf[15]
names = ['act+damp', 'body acc+kinetic', 'joint apply', 'body pos(+vproj)', 'contact pos',
         'body cpos+vproj', 'contact vel', 'body cvel', '-', 'tail']
tot = v.sum()
print('samples', n, 'cycles/wave/step', tot / max(n, 1))
for i, nm in enumerate(names):
  if v[i]:
    print(f'{nm:20s} {100 * v[i] / tot:5.1f}%  {v[i] / max(n, 1):9.0f} cyc')
k = np.array(buf[10:15], dtype=np.float64)
kn = ['prologue (consts, QP/act loads)', 'pbd step', 'observation', 'reward/metrics', 'epilogue (stores)']
kt = k.sum()
print('kernel cycles/wave/step', kt / max(n, 1))
for i, nm in enumerate(kn):
  print(f'{nm:32s} {100 * k[i] / kt:5.1f}%  {k[i] / max(n, 1):9.0f} cyc')
