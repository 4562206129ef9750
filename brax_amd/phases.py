"""Standalone PBD phase kernels on structure-of-arrays batches.

The fused env step keeps state on chip; these entry points run one phase of
`_pbd_step` over an SoA batch in HBM (the integrator and
collider kernels measured against the 8 TB/s roofline on their own):

    soa = to_soa(qp)                     # (13, N, B) fp32: pos|rot|vel|ang planes
    kinetic(sys, soa, out)               # Euler.kinetic          integrators.py:50-68
    update_acc(sys, soa, dp, out)        # Euler.update(acc_p=dp)  integrators.py:85-93
    velocity_projection(sys, soa, prev, out)   #                   integrators.py:122-146
    capsule_plane(sys, soa) -> (10, R, B)      # colliders.py:744-759
"""
import ctypes as C

import torch

from brax_amd import _native
from brax_amd.base import QP

KINETIC, UPDATE_ACC, VPROJ = 0, 1, 2
# algorithmic HBM bytes per body / per contact
BYTES = {KINETIC: 80, UPDATE_ACC: 72, VPROJ: 96, 'capsule_plane': 120}


def _stream(device):
  return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def to_soa(qp: QP):
  """(B,N,·) QP -> (13, N, B) contiguous planes (env fastest)."""
  t = torch.cat([qp.pos, qp.rot, qp.vel, qp.ang], -1)  # (B, N, 13)
  return t.permute(2, 1, 0).contiguous()


def from_soa(soa):
  """(13, N, B) planes -> QP of (B, N, ·) tensors."""
  t = soa.permute(2, 1, 0)
  return QP(pos=t[..., 0:3], rot=t[..., 3:7], vel=t[..., 7:10], ang=t[..., 10:13])


def _check(sys_, soa):
  if soa.dtype != torch.float32 or not soa.is_cuda or not soa.is_contiguous():
    raise ValueError('SoA planes must be a contiguous float32 device tensor')
  if soa.shape[1] != sys_.num_bodies or soa.shape[2] % 4:
    raise ValueError('SoA must be (fields, N, B) with B % 4 == 0')
  return soa.shape[2], soa.shape[1] * soa.shape[2]


def _phase(sys_, which, soa, aux, out):
  B, plane = _check(sys_, soa)
  if out is None:
    out = soa.clone()
  aux_ptr, aux_plane = None, 0
  if aux is not None:
    _check(sys_, aux)
    aux_ptr, aux_plane = C.c_void_p(aux.data_ptr()), aux.shape[1] * aux.shape[2]
  _native.check(_native.lib().bx_phase(sys_._h, which, B, plane, C.c_void_p(soa.data_ptr()),
                                       C.c_void_p(out.data_ptr()), aux_ptr, aux_plane,
                                       _stream(sys_.device)))
  return out


def kinetic(sys_, soa, out=None):
  return _phase(sys_, KINETIC, soa, None, out)


def update_acc(sys_, soa, dp, out=None):
  """dp: (6, N, B) planes of acceleration-level dP (vel xyz, ang xyz)."""
  return _phase(sys_, UPDATE_ACC, soa, dp, out)


def velocity_projection(sys_, soa, prev, out=None):
  return _phase(sys_, VPROJ, soa, prev, out)


def capsule_plane(sys_, soa, out=None):
  """Contacts of every capsule-plane row: (10, R, B) = pos, vel, normal, pen."""
  B, plane = _check(sys_, soa)
  R = sys_.num_rows
  if out is None:
    out = torch.zeros((10, R, B), dtype=torch.float32, device=soa.device)
  _native.check(_native.lib().bx_phase_capsule_plane(
      sys_._h, B, plane, C.c_void_p(soa.data_ptr()), C.c_void_p(out.data_ptr()), R * B,
      _stream(sys_.device)))
  return out
