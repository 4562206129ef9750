"""Per-step conditioning probe of a golden trajectory (diagnostic, CPU only).

For every step t of `traj_<name>`: the fp32 oracle builds' normwise position
error against the float64 golden, and the float64 restatement's own response
to fp32-ulp relative input noise (6e-8). A step where the second is large is
ill-conditioned in float64 itself: any fp32 execution, the reference's jit
included, lands anywhere within that spread.

  python tests/diag/cond_probe.py box_box [n_samples]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from oracle import oracle as ol  # noqa: E402
from tests.conftest import golden  # noqa: E402
from tests.helpers import compiled, normwise  # noqa: E402


def main():
  name = sys.argv[1]
  n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
  d, rd = compiled(name)[1:3]
  T = golden('traj_' + name)
  o64 = ol.Oracle(d, rd, np.float64)
  os32 = [ol.Oracle(d, rd, np.float32, safe_guard=True, fma=f) for f in (False, True)]
  rng = np.random.default_rng(0)
  for t in range(T['action'].shape[0]):
    q, a, ref = T['qp'][t], T['action'][t], T['qp'][t + 1]
    e32 = max(normwise(o.system_step(q.astype(np.float32), a.astype(np.float32))[0][..., 0:3],
                       ref[..., 0:3]).max() for o in os32)
    c = [normwise(o64.system_step(q * (1 + rng.uniform(-6e-8, 6e-8, q.shape)), a)[0][..., 0:3],
                  ref[..., 0:3]).max() for _ in range(n)]
    print(f'{t:3d} e32 {e32:.2e}  f64 response to 6e-8 noise: max {max(c):.2e} '
          f'median {np.median(c):.2e} frac>1e-5 {np.mean(np.array(c) > 1e-5):.2f}')


if __name__ == '__main__':
  main()
