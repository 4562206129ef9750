"""Ant Mountain(4) System.step at 2048 envs across item-loop kernel variants.

    python tools/mountain_ab.py [lanes:mode ...]   (default: 256:3 256:0 64:0)

For NearNeighbors cutoff 0 and 36: steps a warmed state once per kernel
variant (threads per env : mode, 0 item loops, 3 MULTI), reports each
variant's largest normwise difference from the first (0 = bit-equal), then
times 20 steps each (HIP events on the launch stream).
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
  variants = [tuple(int(y) for y in x.split(':')) for x in sys.argv[1:]] or [(256, 3), (256, 0), (64, 0)]
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
    for L, mode in variants:
      _native.check(_native.lib().bx_system_set_variant(sys_._h, L, mode))  # pylint: disable=protected-access
      q1, info = sys_.step(qp, act)
      got = torch.cat([q1.pos.flatten(), q1.rot.flatten(), q1.vel.flatten(), q1.ang.flatten(),
                       info.contact_penetration.flatten()]).cpu()
      diff = None
      if ref is None:
        ref = got
      else:
        diff = float((got - ref).abs().max() / ref.abs().max().clamp(min=1.0))
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
      key = f'L{L}m{mode}'
      res[key] = {'ms_per_step': ms, 'steps_per_s': B / (ms * 1e-3), 'normwise_diff_to_first': diff}
      print(cutoff, key, res[key], flush=True)
    out[f'cutoff{cutoff}'] = res
  print(json.dumps(out))


if __name__ == '__main__':
  main()
