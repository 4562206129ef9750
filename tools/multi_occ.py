"""Ant Mountain(4) System.step time against the batch (diagnostic): how many
MULTI workgroups a CU holds at once shows as the batch past which the step
time grows with it (256 CUs: one env per CU per 256 envs).

    python tools/multi_occ.py [cutoff] [batches ...]   (default 0; 256 512 768 1024 1536 2048)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import brax_amd  # noqa: E402
from brax_amd.envs.mountain import ant_mountain_config  # noqa: E402


def main():
  cutoff = int(sys.argv[1]) if len(sys.argv) > 1 else 0
  batches = [int(x) for x in sys.argv[2:]] or [256, 512, 768, 1024, 1536, 2048]
  dev = torch.device('cuda', 0)
  cfg = ant_mountain_config(4)
  cfg.collider_cutoff = cutoff
  sys_ = brax_amd.System(cfg, device=dev)
  print('lib', os.environ.get('BRAX_AMD_LIB', 'default'), 'package', brax_amd.__file__, 'lanes', sys_.lanes,
        flush=True)
  qp0 = sys_.default_qp()
  for B in batches:
    qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                       for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
    act = torch.rand((B, sys_.action_size), device=dev, generator=torch.Generator(dev).manual_seed(0)) * 2 - 1
    st = [qp]
    for _ in range(5):
      st[0] = sys_.step(st[0], act)[0]
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    a.record()
    for _ in range(n):
      st[0] = sys_.step(st[0], act)[0]
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / n
    print(f'cutoff {cutoff} B {B:5d}: {us:8.1f} us/step  {B / us:6.2f} M steps/s', flush=True)


if __name__ == '__main__':
  main()
