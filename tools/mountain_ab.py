"""Ant Mountain(4) System.step at 2048 envs across item-loop kernel variants.

    python tools/mountain_ab.py [lanes ...]      (default: 64 128 256)

For NearNeighbors cutoff 0 and 36: steps a warmed state once per variant
(lanes per env; mode 0), checks every variant's output bit for bit against
the first, then times 20 steps each (HIP events on the launch stream).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import brax_amd  # noqa: E402
from brax_amd import _native  # noqa: E402
from brax_amd.envs.mountain import ant_mountain_config  # noqa: E402


def main():
  lanes = [int(x) for x in sys.argv[1:]] or [64, 128, 256]
  dev = torch.device('cuda', 0)
  B = 2048
  out = {}
  for cutoff in (0, 36):
    cfg = ant_mountain_config(4)
    cfg.collider_cutoff = cutoff
    sys_ = brax_amd.System(cfg, device=dev)
    qp0 = sys_.default_qp()
    qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                       for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
    g = torch.Generator(device=dev).manual_seed(cutoff)
    act = torch.rand((B, sys_.action_size), device=dev, generator=g) * 2 - 1
    for _ in range(5):  # a state with contacts in flight
      qp, _ = sys_.step(qp, act)
    ref = None
    res = {'default_lanes': sys_.lanes, 'rows': sys_.num_rows}
    for L in lanes:
      _native.check(_native.lib().bx_system_set_variant(sys_._h, L, 0))  # pylint: disable=protected-access
      q1, info = sys_.step(qp, act)
      got = torch.cat([q1.pos.flatten(), q1.rot.flatten(), q1.vel.flatten(), q1.ang.flatten(),
                       info.contact_penetration.flatten()]).cpu()
      same = None
      if ref is None:
        ref = got
      else:
        same = bool(torch.equal(got.view(torch.int32), ref.view(torch.int32)))
      st = [qp]

      def one():
        st[0], _ = sys_.step(st[0], act)
      for _ in range(3):
        one()
      torch.cuda.synchronize()
      a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      a.record()
      n = 20
      for _ in range(n):
        one()
      b.record()
      torch.cuda.synchronize()
      ms = a.elapsed_time(b) / n
      res[f'L{L}'] = {'ms_per_step': ms, 'steps_per_s': B / (ms * 1e-3), 'bit_equal_to_first': same}
      print(cutoff, L, res[f'L{L}'], flush=True)
    out[f'cutoff{cutoff}'] = res
  print(json.dumps(out))


if __name__ == '__main__':
  main()
