"""Ant Mountain(4) kernel variants vs the float64 oracle (diagnostic).

At tools/mountain_ab.py's state (2048 envs, default qp, 5 steps of a fixed
U[-1,1] action), steps once with each kernel variant and prints, per QP
field, the largest normwise error on 16 sampled envs of each variant and of
the fp32 oracle builds (plain / FMA, exact input + 7 ulp-perturbed copies)
against the float64 oracle.

  python tests/diag/mountain_variants.py [cutoff]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import brax_amd  # noqa: E402
from brax_amd import _native  # noqa: E402
from brax_amd.compiler import compile_reset, compile_system  # noqa: E402
from brax_amd.envs.mountain import ant_mountain_config  # noqa: E402
from oracle import oracle as ol  # noqa: E402
from tests.helpers import QP_FIELDS, normwise  # noqa: E402


def main():
  cutoff = int(sys.argv[1]) if len(sys.argv) > 1 else 0
  dev = torch.device('cuda', 0)
  cfg = ant_mountain_config(4)
  cfg.collider_cutoff = cutoff
  sys_ = brax_amd.System(cfg, device=dev)
  B = 2048
  q0 = sys_.default_qp()
  qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                     for t in (q0.pos, q0.rot, q0.vel, q0.ang)))
  g = torch.Generator(device=dev).manual_seed(cutoff)
  act = torch.rand((B, sys_.action_size), device=dev, generator=g) * 2 - 1
  for _ in range(5):
    qp, _ = sys_.step(qp, act)
  idx = np.random.default_rng(3).choice(B, 16, replace=False)
  qp_in = qp.numpy()[idx]
  an = act.cpu().numpy()[idx].astype(np.float64)
  vc, d, meta = compile_system(cfg)
  rd = compile_reset(vc, meta['body_index'])
  ref, _ = ol.Oracle(d, rd, np.float64, safe_guard=True).system_step(qp_in, an)
  rows = {}
  for L, mode in ((256, 3), (256, 0), (64, 0)):
    _native.check(_native.lib().bx_system_set_variant(sys_._h, L, mode))  # pylint: disable=protected-access
    out, _ = sys_.step(qp, act)
    got = out.numpy()[idx]
    rows[f'L{L}m{mode}'] = {f: float(normwise(got[..., sl], ref[..., sl]).max())
                            for f, sl in QP_FIELDS.items()}
  rng = np.random.default_rng(1234)
  e32 = {f: 0.0 for f in QP_FIELDS}
  for fma in (False, True):
    o = ol.Oracle(d, rd, np.float32, safe_guard=True, fma=fma)
    for k in range(8):
      q = qp_in if k == 0 else qp_in * (1 + rng.uniform(-6e-8, 6e-8, qp_in.shape))
      out, _ = o.system_step(q.astype(np.float32), an.astype(np.float32))
      for f, sl in QP_FIELDS.items():
        e32[f] = max(e32[f], float(normwise(out[..., sl], ref[..., sl]).max()))
  rows['fp32 envelope'] = e32
  for k, v in rows.items():
    print(f'{k:>14}', ' '.join(f'{f}={x:.3e}' for f, x in v.items()), flush=True)


if __name__ == '__main__':
  main()
