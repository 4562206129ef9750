"""Diagnostic: per-wave cycle spread of the single-mode env step (BX_STAMPS
build, BRAX_AMD_LIB=...): the kernel lasts as long as its slowest wave, so
the spread of the per-wave totals (one workgroup = one wave of 4 envs)
tells how much of the kernel time is data-dependent imbalance.

    BRAX_AMD_LIB=brax_amd/_lib_stamps/libbrax_amd.so python tools/wave_spread.py halfcheetah
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import _native, envs  # noqa: E402

dev = torch.device('cuda', 0)
name = sys.argv[1] if len(sys.argv) > 1 else 'halfcheetah'
B = 4096
env = envs.create(name, batch_size=B, episode_length=1000, device=dev)
st = env.reset(np.array([0, 1], np.uint32))
lib = _native.lib()
buf = (C.c_ulonglong * (4096 * 16))()
g = torch.Generator(device='cpu').manual_seed(0)
for k in range(40):
  if k == 20:
    torch.cuda.synchronize()
    _native.check(lib.bx_debug_stamps(buf, 1))
  a = (torch.rand((B, env.action_size), generator=g) * 2 - 1).to(dev)
  st = env.step(st, a)
torch.cuda.synchronize()
_native.check(lib.bx_debug_stamps(buf, 4))
w = np.array(buf, dtype=np.float64).reshape(4096, 16)[:B // 4]
n = w[:, 15]
pbd = w[:, :10].sum(1) / np.maximum(n, 1)
kern = w[:, 10:15].sum(1) / np.maximum(n, 1)
out = {'env': name, 'waves': int((n > 0).sum()), 'steps_per_wave': float(n.max()),
       'kernel_cycles_per_step': {'mean': kern.mean(), 'p50': float(np.median(kern)),
                                  'p99': float(np.percentile(kern, 99)), 'max': kern.max()},
       'pbd_cycles_per_step': {'mean': pbd.mean(), 'max': pbd.max()},
       'phase_mean_vs_slowest_wave': {
           str(k): [w[:, k].mean() / max(n.max(), 1), w[int(kern.argmax()), k] / max(n.max(), 1)]
           for k in range(10)}}
print(json.dumps(out))
