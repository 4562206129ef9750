"""`brax/math.py` on torch tensors (batched over leading axes; quaternions
are wxyz). Used by the host-side env layer; the kernels have their own
device versions in csrc/pbd_math.h."""
import math as _m

import torch

from brax_amd.base import rotate  # noqa: F401  (math.py:25-40)


def quat_inv(q):
  """`math.py:190-199`."""
  return q * torch.tensor([1., -1., -1., -1.], dtype=q.dtype, device=q.device)


def inv_rotate(vec, quat):
  """`math.py:43-53`: rotate by the inverse of a unit quaternion."""
  return rotate(vec, quat_inv(quat))


def quat_mul(u, v):
  """`math.py:133-154`: Hamilton product."""
  uw, ux, uy, uz = u.unbind(-1)
  vw, vx, vy, vz = v.unbind(-1)
  return torch.stack([
      uw * vw - ux * vx - uy * vy - uz * vz,
      uw * vx + ux * vw + uy * vz - uz * vy,
      uw * vy - ux * vz + uy * vw + uz * vx,
      uw * vz + ux * vy - uy * vx + uz * vw], -1)


def safe_arcsin(x):
  """`jumpy.py:323-334` (value path): arcsin of x clipped into [-1, 1]."""
  return torch.arcsin(torch.clamp(x, -1., 1.))


def quat_to_euler(q):
  """`math.py:80-91`: x-y'-z'' Tait-Bryan angles in radians, (..., 3)."""
  w, x, y, z = q.unbind(-1)
  zz = torch.atan2(-2 * x * y + 2 * w * z, x * x + w * w - z * z - y * y)
  yy = safe_arcsin(torch.clamp(2 * x * z + 2 * w * y, -1., 1.))
  xx = torch.atan2(-2 * y * z + 2 * w * x, z * z - y * y - x * x + w * w)
  return torch.stack([xx, yy, zz], -1)


PI = _m.pi
