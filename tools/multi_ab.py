"""Ant Mountain(4) System.step at 2048 envs (BASELINE configs[4]) on the
library BRAX_AMD_LIB names: us per step (HIP events over back-to-back steps
on the launch stream) for NearNeighbors cutoff 0 / 36, Info on / off; one
JSON line (tools/multi_ab.sh runs it per build, interleaved)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import brax_amd  # noqa: E402
from brax_amd.envs.mountain import ant_mountain_config  # noqa: E402


def main():
  dev = torch.device('cuda', 0)
  B, n = 2048, 30
  out = {'lib': os.environ.get('BRAX_AMD_LIB', 'brax_amd/_lib'),
         'warm_steps': int(os.environ.get('BX_MULTI_WARM', '10')),
         'lanes': os.environ.get('BX_MULTI_LANES', 'default')}
  for cutoff in (0, 36):
    cfg = ant_mountain_config(4)
    cfg.collider_cutoff = cutoff
    sys_ = brax_amd.System(cfg, device=dev)
    if os.environ.get('BX_MULTI_LANES'):
      from brax_amd import _native
      _native.check(_native.lib().bx_system_set_variant(sys_._h, int(os.environ['BX_MULTI_LANES']), 3))
    qp0 = sys_.default_qp()
    qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                       for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
    g = torch.Generator(device=dev).manual_seed(cutoff)
    act = torch.rand((B, sys_.action_size), device=dev, generator=g) * 2 - 1
    for info in (True, False):
      q = qp
      for _ in range(int(os.environ.get('BX_MULTI_WARM', '10'))):
        q, _ = sys_.step(q, act, info=info)
      torch.cuda.synchronize()
      a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      a.record()
      for _ in range(n):
        q, _ = sys_.step(q, act, info=info)
      b.record()
      torch.cuda.synchronize()
      us = a.elapsed_time(b) * 1e3 / n
      out[f'cutoff{cutoff}_{"info" if info else "noinfo"}'] = {'us': round(us, 1),
                                                               'M_steps_per_s': round(B / us, 3)}
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  main()
