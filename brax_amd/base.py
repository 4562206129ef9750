"""State containers: QP / P / Q / Info (`brax/physics/base.py:28-153`).

Same field names, shapes and arithmetic as the reference (rot is wxyz), but
the leaves are torch tensors living in HBM. A batch has a leading env axis:
pos (B,N,3), rot (B,N,4), vel (B,N,3), ang (B,N,3).

States produced by brax_amd are strided views of one packed (B,N,16) fp32
buffer (pos 0:3, rot 3:7, vel 7:10, ang 10:13), so they reach the kernels
without copies; any user-built QP of contiguous fields works too.
"""
import dataclasses
from typing import Any

import torch


def _add(a, b):
  return a + b


@dataclasses.dataclass(frozen=True)
class Q:
  """Coordinates: position and rotation (`base.py:28-47`)."""
  pos: Any
  rot: Any

  def __add__(self, o):
    if isinstance(o, P):
      return QP(self.pos, self.rot, o.vel, o.ang)
    if isinstance(o, Q):
      return Q(self.pos + o.pos, self.rot + o.rot)
    if isinstance(o, QP):
      return QP(self.pos + o.pos, self.rot + o.rot, o.vel, o.ang)
    raise ValueError('add only supported for P, Q, QP')

  def replace(self, **kw):
    return dataclasses.replace(self, **kw)


@dataclasses.dataclass(frozen=True)
class P:
  """Time derivatives: velocity and angular velocity (`base.py:50-72`)."""
  vel: Any
  ang: Any

  def __add__(self, o):
    if isinstance(o, P):
      return P(self.vel + o.vel, self.ang + o.ang)
    if isinstance(o, Q):
      return QP(o.pos, o.rot, self.vel, self.ang)
    if isinstance(o, QP):
      return QP(o.pos, o.rot, self.vel + o.vel, self.ang + o.ang)
    raise ValueError('add only supported for P, Q, QP')

  def __mul__(self, o):
    return P(self.vel * o, self.ang * o)

  def replace(self, **kw):
    return dataclasses.replace(self, **kw)


@dataclasses.dataclass(frozen=True)
class QP:
  """Position, rotation, velocity, angular velocity (`base.py:75-133`)."""
  pos: Any
  rot: Any
  vel: Any
  ang: Any

  def __add__(self, o):
    if isinstance(o, P):
      return QP(self.pos, self.rot, self.vel + o.vel, self.ang + o.ang)
    if isinstance(o, Q):
      return QP(self.pos + o.pos, self.rot + o.rot, self.vel, self.ang)
    if isinstance(o, QP):
      return QP(self.pos + o.pos, self.rot + o.rot, self.vel + o.vel,
                self.ang + o.ang)
    raise ValueError('add only supported for P, Q, QP')

  def __mul__(self, o):
    return QP(self.pos * o, self.rot * o, self.vel * o, self.ang * o)

  def replace(self, **kw):
    return dataclasses.replace(self, **kw)

  @classmethod
  def zero(cls, shape=(), device=None):
    z = torch.zeros(shape + (16,), dtype=torch.float32, device=device)
    z[..., 3] = 1.0
    return packed_view(z)

  def __getitem__(self, idx):
    return QP(self.pos[idx], self.rot[idx], self.vel[idx], self.ang[idx])

  @property
  def shape(self):
    return tuple(self.pos.shape[:-1])

  def to_world(self, rpos):
    """World position and velocity of a body-frame point (`base.py:112-125`)."""
    off = rotate(torch.as_tensor(rpos, dtype=self.rot.dtype, device=self.rot.device),
                 self.rot)
    return self.pos + off, self.vel + torch.cross(self.ang, off, dim=-1)

  def world_velocity(self, pos):
    return self.vel + torch.cross(self.ang, pos - self.pos, dim=-1)

  def numpy(self):
    """(…, N, 13) float64 numpy array: pos | rot | vel | ang."""
    import numpy as np  # pylint: disable=import-outside-toplevel
    return np.concatenate([t.detach().double().cpu().numpy() for t in
                           (self.pos, self.rot, self.vel, self.ang)], -1)


@dataclasses.dataclass(frozen=True)
class Info:
  """Auxiliary step data (`base.py:136-153`)."""
  contact: P
  joint: Any
  actuator: P
  contact_pos: Any
  contact_normal: Any
  contact_penetration: Any
  # beyond the reference's fields: the NearNeighbors cell i * U + j behind
  # each contact row (the `idx` of `top_k`, colliders.py:84), -1 for Pairs
  # rows; None for systems without culled collider groups
  contact_cell: Any = None

  def replace(self, **kw):
    return dataclasses.replace(self, **kw)


def rotate(vec, quat):
  """`brax/math.py:25-40` on torch tensors (broadcasting over leading axes)."""
  s, u = quat[..., :1], quat[..., 1:]
  r = 2 * ((u * vec).sum(-1, keepdim=True) * u) + (s * s - (u * u).sum(-1, keepdim=True)) * vec
  return r + 2 * s * torch.cross(u.expand_as(r), vec.expand_as(r), dim=-1)


class PackedQP(QP):
  """A QP over one packed (…, N, 16) fp32 buffer (pos 0:3, rot 3:7,
  vel 7:10, ang 10:13). Its field views are built on first access: the
  kernels take the buffer itself, so a state that is only stepped never
  builds them (each torch view costs ~1 µs of host time per step). Behaves
  as a QP otherwise; `replace` returns a plain QP."""

  def __new__(cls, buf=None, **fields):
    if fields:  # dataclasses.replace(packed_qp, ...) rebuilds by fields
      return QP(**fields)
    return object.__new__(cls)

  def __init__(self, buf=None, **fields):  # pylint: disable=super-init-not-called
    del fields
    object.__setattr__(self, '_buf', buf)

  def _fields(self):
    f = self.__dict__.get('_f')
    if f is None:
      f = torch.split(self._buf, [3, 4, 3, 3, 3], -1)[:4]
      object.__setattr__(self, '_f', f)
    return f

  pos = property(lambda self: self._fields()[0])
  rot = property(lambda self: self._fields()[1])
  vel = property(lambda self: self._fields()[2])
  ang = property(lambda self: self._fields()[3])

  def replace(self, **kw):
    return QP(**{k: kw.get(k, getattr(self, k)) for k in ('pos', 'rot', 'vel', 'ang')})

  @property
  def shape(self):
    return tuple(self._buf.shape[:-1])


def packed_view(buf):
  """QP whose fields are views of a (…, N, 16) fp32 buffer."""
  return PackedQP(buf)


def packed_buffer(qp):
  """The (…, N, 16) buffer behind a packed QP, or None."""
  if type(qp) is PackedQP:
    return qp._buf  # pylint: disable=protected-access
  base = qp.pos
  if base._base is None:  # pylint: disable=protected-access
    return None
  buf = base._base  # pylint: disable=protected-access
  if (buf.dim() == qp.pos.dim() and buf.shape[-1] == 16 and
      qp.pos.data_ptr() == buf.data_ptr() and
      qp.rot.data_ptr() == buf.data_ptr() + 12 and
      qp.vel.data_ptr() == buf.data_ptr() + 28 and
      qp.ang.data_ptr() == buf.data_ptr() + 40):
    return buf
  return None


def qp_from_numpy(a, device):
  """(…, N, 13) array -> packed QP on `device`."""
  t = torch.as_tensor(a, dtype=torch.float32)
  buf = torch.zeros(t.shape[:-1] + (16,), dtype=torch.float32)
  buf[..., :13] = t
  return packed_view(buf.to(device))
