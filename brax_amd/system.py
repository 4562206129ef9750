"""`brax.System` on MI355X (`brax/physics/system.py:46-340`).

    sys = brax_amd.System(config)            # text proto or brax_amd.Config
    qp = sys.default_qp()                    # QP (N,·) on the device
    qp, info = sys.step(qp, act)             # batched if qp has a leading axis

`step` runs the fused PBD kernel (`bx_system_step`); `default_qp` and `info`
run their own kernels. Every call is stream-ordered on torch's current stream.
There is no CPU fallback: without a GPU or the built library the constructor
raises.
"""
import ctypes as C

import numpy as np
import torch

from brax_amd import _native
from brax_amd import abi
from brax_amd import compiler
from brax_amd import config as cfgmod
from brax_amd.base import Info, P, PackedQP, QP, packed_view


try:
  _raw_stream = torch._C._cuda_getCurrentRawStream  # pylint: disable=protected-access
except AttributeError:  # pragma: no cover
  _raw_stream = None


def _stream(device_index=None):
  """The caller's current HIP stream on `device_index` (stream-ordered ABI,
  SURVEY §8(b)); every System call passes its own device's index."""
  if _raw_stream is not None:
    return C.c_void_p(_raw_stream(torch.cuda.current_device() if device_index is None
                                  else device_index))
  return C.c_void_p(torch.cuda.current_stream(device_index).cuda_stream)


def _field(t, batched):
  if t.dtype != torch.float32 or not t.is_cuda:
    raise TypeError('QP fields must be float32 device tensors')
  if t.stride(-1) != 1:
    raise ValueError('QP fields need a unit innermost stride')
  f = abi.BxField()
  f.ptr = t.data_ptr()
  f.env_stride = t.stride(0) if batched else 0
  f.body_stride = t.stride(-2)
  return f


def qp_struct(qp, batched):
  """bx_qp view of a QP. Batched structs are cached on the (frozen) QP: its
  fields cannot be re-bound, so the pointers and strides stay valid."""
  if batched and type(qp) is PackedQP and qp._buf.dim() == 3:  # pylint: disable=protected-access
    # the packed buffer itself: no field views
    s = qp.__dict__.get('_bxs')
    if s is not None:
      return s
    buf = qp._buf  # pylint: disable=protected-access
    if buf.dtype != torch.float32 or not buf.is_cuda or not buf.is_contiguous():
      raise TypeError('QP fields must be float32 device tensors')
    base, es = buf.data_ptr(), buf.stride(0)
    s = abi.BxQP()
    for name, off in (('pos', 0), ('rot', 3), ('vel', 7), ('ang', 10)):
      f = getattr(s, name)
      f.ptr = base + 4 * off
      f.env_stride = es
      f.body_stride = 16
    object.__setattr__(qp, '_bxs', s)
    return s
  if batched:
    s = qp.__dict__.get('_bxs')
    # (a copied QP carries the attribute over: re-check the pointers)
    if (s is not None and s.pos.ptr == qp.pos.data_ptr() and s.rot.ptr == qp.rot.data_ptr()
        and s.vel.ptr == qp.vel.data_ptr() and s.ang.ptr == qp.ang.data_ptr()):
      return s
  s = abi.BxQP()
  s.pos = _field(qp.pos, batched)
  s.rot = _field(qp.rot, batched)
  s.vel = _field(qp.vel, batched)
  s.ang = _field(qp.ang, batched)
  if batched:
    object.__setattr__(qp, '_bxs', s)
  return s


class JointGroup:
  """One entry of `System.joints` (`joints.get` groups joints by dof,
  joints.py:418-474); only `angle_vel` is needed on the host side."""

  def __init__(self, sys_, lo, hi, dof, names, free):
    self._sys, self._lo, self._hi = sys_, lo, hi
    self.dof, self.names, self.free_dofs = dof, list(names), free

  def angle_vel(self, qp):
    """`Joint.angle_vel` (joints.py:197-226): angles and velocities of this
    group's dofs, (..., n) each, free dofs only for sphericalised groups."""
    a, v = self._sys.joint_angle_vel(qp)
    return a[..., self._lo:self._hi], v[..., self._lo:self._hi]


class Body:
  """Per-body constants (`bodies.py:25-59`): mass and INVERSE inertia."""

  def __init__(self, desc, index):
    self.mass = desc['body_mass'].copy()
    self.inertia = desc['body_inv_inertia'].copy()
    self.index = dict(index)
    self.idx = np.arange(len(self.mass))


class System:
  """A brax system compiled for the MI355X kernels."""

  def __init__(self, config, device=None):
    if isinstance(config, str):
      config = cfgmod.parse(config)
    self.config, self.desc, meta = compiler.compile_system(config)
    self._body_index = meta['body_index']
    self.reset_desc = compiler.compile_reset(self.config, self._body_index)
    self.num_bodies = int(self.desc['n_bodies'])
    self.num_joints = len(self.config.joints)
    self.num_joint_dof = meta['num_joint_dof']
    self.num_forces_dof = meta['num_forces_dof']
    self.num_actuators = len(self.config.actuators)
    self.action_size = meta['action_size']
    self.num_rows = len(self.desc["row_group"])  # contact rows (every candidate cell)
    self.num_contacts = abi.info_rows(self.desc)  # Info contact rows (system.py:36-43)
    self._culled = bool((np.asarray(self.desc.get('col_cutoff', [0])) > 0).any())
    self.body = Body(self.desc, meta['body_index'])
    self.joint_groups = meta['joint_groups']
    self.joints = []
    lo = 0
    for dof, names, free in self.joint_groups:
      n = sum(free) if free is not None else dof * len(names)
      self.joints.append(JointGroup(self, lo, lo + n, dof, names, free))
      lo += n
    if device is None:
      if not torch.cuda.is_available():
        raise _native.NativeError('brax_amd.System needs a GPU (no CPU fallback)')
      device = torch.device('cuda', torch.cuda.current_device())
    self.device = torch.device(device)
    if self.device.type != 'cuda':
      raise _native.NativeError('brax_amd runs on MI355X devices only')
    self._h = self._create(self.reset_desc)
    self._default_h = {0: self._h}  # one handle per config.defaults index used
    self.lanes = _native.lib().bx_system_lanes(self._h)

  @property
  def env_lanes(self):
    """Threads per env of the Env.step / rollout kernels (bx_system_env_lanes):
    the step kernels' `lanes`."""
    return _native.lib().bx_system_env_lanes(self._h)

  @property
  def lds_bytes(self):
    """LDS bytes per workgroup of the System.step kernel (bx_system_lds_bytes)."""
    return _native.lib().bx_system_lds_bytes(self._h)

  @staticmethod
  def plan(config):
    """The kernel plan `config` compiles to, on the host without a device
    (bx_system_plan): {'mode': 1 SINGLE / 3 MULTI / 0 item loops, 'lanes':
    threads per env, 'lds_bytes': the System.step kernel's LDS per workgroup,
    'envs_per_cu_by_lds': what 160 KB of LDS holds, 'envs_per_cu_by_registers':
    what the register file holds (MULTI: the kernel is built for two waves per
    SIMD, 256 registers, so eight waves per CU: four 128-thread envs or two
    256-thread ones; None where not fixed by the build), 'envs_per_cu': the
    smaller of the two, i.e. what runs}."""
    vc, desc, meta = compiler.compile_system(config)
    rdesc = compiler.compile_reset(vc, meta['body_index'])
    cd, keep = abi.make_desc(desc)
    rd, keep_r = abi.make_reset_desc(rdesc, meta['num_joint_dof'])
    mode, lanes, lds = C.c_int32(), C.c_int32(), C.c_int32()
    _native.check(_native.lib().bx_system_plan(C.byref(cd), C.byref(rd), C.byref(mode),
                                               C.byref(lanes), C.byref(lds)))
    del keep, keep_r
    per_wg = lds.value
    envs_per_wg = max(64 // lanes.value, 1)
    by_lds = (160 * 1024 // per_wg) * envs_per_wg if per_wg else None
    # system_step_multi_kernel<L>: amdgpu_waves_per_eu(2) (pbd_kernels.hip):
    # 256 registers, two waves per SIMD, eight per CU, L / 64 per env
    by_regs = 8 // (lanes.value // 64) if mode.value == 3 else None
    runs = min(x for x in (by_lds, by_regs) if x is not None) if (by_lds or by_regs) else None
    return {'mode': mode.value, 'lanes': lanes.value, 'lds_bytes': per_wg,
            'envs_per_cu_by_lds': by_lds, 'envs_per_cu_by_registers': by_regs,
            'envs_per_cu': runs}

  def _create(self, reset_desc):
    cd, keep = abi.make_desc(self.desc)
    rd, keep_r = abi.make_reset_desc(reset_desc, self.num_joint_dof)
    h = C.c_void_p()
    _native.check(_native.lib().bx_system_create(C.byref(cd), C.byref(rd),
                                                 self.device.index or 0, C.byref(h)))
    del keep, keep_r
    return h

  def _default_handle(self, default_index):
    """Handle whose reset descriptor is `config.defaults[default_index]`
    (system.py:112-242 reads the default by index; an index past the list
    means no default, as there)."""
    if default_index not in self._default_h:
      self._default_h[default_index] = self._create(
          compiler.compile_reset(self.config, self._body_index, default_index))
    return self._default_h[default_index]

  def __del__(self):
    for h in getattr(self, '_default_h', {}).values():
      if h is not None and h.value:
        try:
          _native.lib().bx_system_destroy(h)
        except Exception:  # pylint: disable=broad-except
          pass

  # ---------------------------------------------------------------- helpers
  def _new_qp(self, lead):
    return packed_view(torch.empty(lead + (self.num_bodies, 16), dtype=torch.float32,
                                   device=self.device))

  def _act(self, act, B):
    if act is None:
      act = torch.zeros((B, self.action_size), dtype=torch.float32, device=self.device)
    act = torch.as_tensor(act, dtype=torch.float32, device=self.device)
    if act.dim() == 1:
      act = act.reshape(1, -1).expand(B, -1) if B > 1 else act.reshape(1, -1)
    if act.dim() != 2 or act.shape[0] != B:
      raise ValueError(f'action shape {tuple(act.shape)} does not match {B} envs')
    # any width: indices are clipped like the reference's jp.take (jumpy.py:151)
    if act.shape[-1] == 0 and (self.num_actuators or self.num_forces_dof):
      raise ValueError('empty action for a system with actuators or forces')
    if act.stride(-1) != 1:
      act = act.contiguous()
    return act

  # ---------------------------------------------------------------- API
  def default_angle(self, default_index: int = 0):
    """`System.default_angle` (system.py:86-110)."""
    a = compiler.default_angle(self.config, default_index)
    return torch.as_tensor(a, dtype=torch.float32, device=self.device)

  def default_qp(self, default_index: int = 0, joint_angle=None, joint_velocity=None):
    """`System.default_qp` (system.py:112-242) on the device.

    joint_angle / joint_velocity may carry a leading batch axis; the result
    then is batched too."""
    if joint_angle is None:
      joint_angle = self.default_angle(default_index)
    ja = torch.as_tensor(joint_angle, dtype=torch.float32, device=self.device)
    batched = ja.dim() == 2
    D = self.num_joint_dof
    if D == 0:
      B = ja.shape[0] if batched else 1
      ja = torch.zeros((B, 0), dtype=torch.float32, device=self.device)
    else:
      ja = ja.reshape(-1, ja.shape[-1]) if batched else ja.reshape(1, -1)
      B = ja.shape[0]
    # the angle vector lists only the dofs with a nonzero limit
    # (system.py:86-110,138-141); the reset tables index that prefix, so
    # rows are padded to the kernel's num_joint_dof stride
    def pad(x):
      if x.shape[1] > D:
        raise ValueError(f'{x.shape[1]} joint dofs given, the system has {D}')
      return torch.nn.functional.pad(x, (0, D - x.shape[1])).contiguous()

    ja = pad(ja)
    if joint_velocity is None:
      jv = torch.zeros_like(ja)
    else:
      jv = pad(torch.as_tensor(joint_velocity, dtype=torch.float32,
                               device=self.device).reshape(B, -1))
    out = self._new_qp((B,))
    qs = qp_struct(out, True)
    _native.check(_native.lib().bx_system_default_qp(
        self._default_handle(default_index), B, C.c_void_p(ja.data_ptr()), C.c_void_p(jv.data_ptr()), C.byref(qs),
        _stream(self.device.index)))
    return out if batched else out[0]

  def step(self, qp: QP, act, info: bool = True):
    """`System.step` (system.py:244-325): (QP, act) -> (QP, Info).

    info=False: (QP, None) -- the step without its Info outputs (the per-body
    contact / actuator sums and the per-row contact_pos / normal /
    penetration), for callers that read only the state, as XLA drops Info
    under jit when the caller ignores it. The state is the same bits; the
    large-scene kernel also skips the contact math of far capsule pairs on
    the step's last collision pass (their rows would only feed Info)."""
    batched = qp.pos.dim() == 3
    B = qp.pos.shape[0] if batched else 1
    act = self._act(act, B)
    lead = (B,) if batched else ()
    out = self._new_qp(lead)
    if not info:
      qi = qp_struct(qp, batched)
      qo = qp_struct(out, batched)
      _native.check(_native.lib().bx_system_step(
          self._h, B, C.byref(qi), C.c_void_p(act.data_ptr()), act.stride(0), act.shape[1],
          C.byref(qo), None, _stream(self.device.index)))
      return out, None
    N, R = self.num_bodies, self.num_contacts
    spring = int(self.desc.get('dynamics_mode', 0)) == abi.DYN_LEGACY_SPRING
    cbuf = torch.empty(lead + (N, 18 if spring else 12), dtype=torch.float32, device=self.device)
    cvel, cang = cbuf[..., 0:3], cbuf[..., 3:6]
    aang = cbuf[..., 9:12]
    avel = cbuf[..., 6:9]
    cpos = torch.empty(lead + (R, 3), dtype=torch.float32, device=self.device)
    cnorm = torch.empty(lead + (R, 3), dtype=torch.float32, device=self.device)
    cpen = torch.empty(lead + (R,), dtype=torch.float32, device=self.device)
    info = abi.BxInfo()
    info.contact_vel = _field(cvel, batched)
    info.contact_ang = _field(cang, batched)
    info.actuator_vel = _field(avel, batched)
    info.actuator_ang = _field(aang, batched)
    if spring:  # Info.joint: accumulated spring dp_j (zero_info under pbd)
      info.joint_vel = _field(cbuf[..., 12:15], batched)
      info.joint_ang = _field(cbuf[..., 15:18], batched)
    cell = None
    if R:
      info.contact_pos = cpos.data_ptr()
      info.contact_normal = cnorm.data_ptr()
      info.contact_penetration = cpen.data_ptr()
      if self._culled:
        cell = torch.empty(lead + (R,), dtype=torch.int32, device=self.device)
        info.contact_cell = cell.data_ptr()
    qi = qp_struct(qp, batched)
    qo = qp_struct(out, batched)
    _native.check(_native.lib().bx_system_step(
        self._h, B, C.byref(qi), C.c_void_p(act.data_ptr()), act.stride(0), act.shape[1],
        C.byref(qo), C.byref(info), _stream(self.device.index)))
    zero = torch.zeros_like(cvel)
    joint = P(cbuf[..., 12:15], cbuf[..., 15:18]) if spring else P(zero, zero)
    return out, Info(contact=P(cvel, cang), joint=joint, actuator=P(avel, aang),
                     contact_pos=cpos, contact_normal=cnorm, contact_penetration=cpen,
                     contact_cell=cell)

  def joint_angle_vel(self, qp: QP):
    """Angles and angular velocities of every joint dof, in joint order
    (`bx_system_joint_angles`): two (B, num_joint_dof) tensors (unbatched QP:
    (num_joint_dof,))."""
    batched = qp.pos.dim() == 3
    B = qp.pos.shape[0] if batched else 1
    D = sum(j._hi - j._lo for j in self.joints)  # pylint: disable=protected-access
    buf = torch.empty((2, B, D), dtype=torch.float32, device=self.device)
    if D:
      qs = qp_struct(qp, batched)
      _native.check(_native.lib().bx_system_joint_angles(
          self._h, B, C.byref(qs), C.c_void_p(buf[0].data_ptr()), C.c_void_p(buf[1].data_ptr()),
          _stream(self.device.index)))
    return (buf[0], buf[1]) if batched else (buf[0, 0], buf[1, 0])

  def info(self, qp: QP):
    """`System.info` (system.py:249-252, 327-340, 377-390): the contact part
    (Collider.apply, the same impulse model in both dynamics modes)."""
    batched = qp.pos.dim() == 3
    B = qp.pos.shape[0] if batched else 1
    lead = (B,) if batched else ()
    cbuf = torch.empty(lead + (self.num_bodies, 6), dtype=torch.float32, device=self.device)
    info = abi.BxInfo()
    info.contact_vel = _field(cbuf[..., 0:3], batched)
    info.contact_ang = _field(cbuf[..., 3:6], batched)
    qi = qp_struct(qp, batched)
    _native.check(_native.lib().bx_system_info(self._h, B, C.byref(qi), C.byref(info),
                                               _stream(self.device.index)))
    zero = torch.zeros_like(cbuf[..., 0:3])
    return Info(contact=P(cbuf[..., 0:3], cbuf[..., 3:6]), joint=P(zero, zero),
                actuator=P(zero, zero), contact_pos=None, contact_normal=None,
                contact_penetration=None)
