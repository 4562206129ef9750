"""Diagnostic: the single-step Env.step kernel's prologue, part by part
(a -DBX_STAMPS -DBX_PSTAMPS build: s_memtime stamps between the prologue's
parts, the pbd phases not stamped), 4,096 envs of argv[1] (default ant).
Cycles per wave and step of: the header / LDS setup, issuing the lane-image
loads, issuing the per-env scalar loads, the state's arrival (every earlier
load's latency: vmcnt is in order) and its LDS copy, the action row, then the
kernel's remaining parts."""
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
n = max(buf[15], 1)
names = {5: 'header + LDS carve / zero', 6: 'lane-image loads issued', 7: 'per-env scalars issued',
         8: 'state arrival + LDS copy', 9: '-', 10: 'action row staged',
         11: 'pbd step', 12: 'observation', 13: 'reward / metrics', 14: 'epilogue (stores)'}
v = {k: buf[k] / n for k in names}
tot = sum(v.values())
print('samples', n, 'cycles/wave/step', tot)
for k, nm in names.items():
  if v[k]:
    print(f'{nm:28s} {100 * v[k] / tot:5.1f}%  {v[k]:9.0f} cyc')
# a -DBX_OSTAMPS build: the observation's parts (slots 0..4, inside slot 12)
sub = {0: 'obs: joint angles', 1: 'obs: centre of mass + sync', 2: 'obs: torso / joint words',
       3: 'obs: per-body loop', 4: 'obs: actuator words'}
for k, nm in sub.items():
  if buf[k]:
    print(f'  {nm:26s} {buf[k] / n:9.0f} cyc')
