"""ctypes front-end of the C restatement (oracle/pbd_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, `__graft_entry__.smoke()` and
bench.py's cpu_baseline leg — never by the `brax_amd` product package.

    o = Oracle(desc, reset_desc, dtype=np.float64)
    qp1, info = o.system_step(qp0, act)          # qp (B,N,13) pos|rot|vel|ang
"""
import ctypes as C
import os
import subprocess

import numpy as np

from brax_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'liboracle.so')

ENV_KIND = {'none': 0, 'ant': 1, 'humanoid': 2, 'halfcheetah': 3, 'humanoidstandup': 4,
            'hopper': 5, 'walker2d': 6, 'inverted_pendulum': 7, 'inverted_double_pendulum': 8,
            'acrobot': 9, 'reacher': 10, 'reacherangle': 11, 'swimmer': 12, 'pusher': 13,
            'ur5e': 14, 'fetch': 15, 'grasp': 16}


def build():
  """make, under a file lock: parallel test workers (pytest -n) would
  otherwise rebuild the same objects concurrently."""
  import fcntl
  os.makedirs(os.path.join(HERE, '_build'), exist_ok=True)
  with open(os.path.join(HERE, '_build', '.lock'), 'w') as lk:
    fcntl.flock(lk, fcntl.LOCK_EX)
    subprocess.run(['make', '-s', '-C', HERE], check=True)


def _load():
  if not os.path.exists(LIB):
    build()
  lib = C.CDLL(LIB)
  return lib


_LIB = None


def lib():
  global _LIB
  if _LIB is None:
    _LIB = _load()
  return _LIB


def _p(a):
  return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
  """C restatement at float64 (checker) or float32 (CPU baseline)."""

  def __init__(self, desc, reset_desc=None, dtype=np.float64, safe_guard=True, fma=False):
    """fma=True (float32 only): the build with a*b+c contracted to fused
    multiply-adds, as XLA's jit and hipcc contract them."""
    self.dtype = np.dtype(dtype)
    self.suf = '_f64' if self.dtype == np.float64 else ('_f32fma' if fma else '_f32')
    self.desc = dict(desc)
    self.cdesc, self._keep = abi.make_desc(self.desc)
    self.N = int(desc['n_bodies'])
    self.R = len(desc['row_group'])
    self.IR = abi.info_rows(self.desc)  # Info contact rows
    self.A = int(desc.get('action_size', 0))
    if reset_desc is not None:
      self.creset, self._keep_r = abi.make_reset_desc(reset_desc,
                                                      desc.get('num_joint_dof'))
    else:
      self.creset = None
    self._fn('oracle_set_safe_norm_guard')(C.c_int(1 if safe_guard else 0))

  def _fn(self, name):
    return getattr(lib(), name + self.suf)

  def _a(self, x):
    return np.ascontiguousarray(np.asarray(x, self.dtype))

  def set_threads(self, n):
    self._fn('oracle_set_threads')(C.c_int(n))

  def max_threads(self):
    return int(self._fn('oracle_max_threads')())

  def _width(self, act):
    """Rows of any width >= 1: indices clip like jp.take (jumpy.py:151)."""
    self._fn('oracle_set_act_width')(C.c_int(act.shape[1]))

  def system_step(self, qp, act):
    qp = self._a(qp)
    B = qp.shape[0]
    act = self._a(act).reshape(B, -1)
    self._width(act)
    out = np.empty_like(qp)
    ic = np.empty((B, self.N, 6), self.dtype)
    ia = np.empty((B, self.N, 6), self.dtype)
    cp = np.empty((B, self.IR, 3), self.dtype)
    cn = np.empty((B, self.IR, 3), self.dtype)
    pen = np.empty((B, self.IR), self.dtype)
    ij = np.empty((B, self.N, 6), self.dtype)
    self._fn('oracle_system_step')(C.byref(self.cdesc), C.c_int64(B), _p(qp), _p(act),
                                   _p(out), _p(ic), _p(ia), _p(cp), _p(cn), _p(pen), _p(ij))
    return out, dict(contact=ic, actuator=ia, contact_pos=cp, contact_normal=cn,
                     contact_penetration=pen, joint=ij)

  def system_info(self, qp):
    qp = self._a(qp)
    B = qp.shape[0]
    ic = np.empty((B, self.N, 6), self.dtype)
    self._fn('oracle_system_info')(C.byref(self.cdesc), C.c_int64(B), _p(qp), _p(ic))
    return ic

  @staticmethod
  def _coef(coef):
    if coef is None:
      return None, None
    c = np.ascontiguousarray(np.asarray(coef, np.float64).reshape(8))
    return c, c.ctypes.data_as(C.POINTER(C.c_double))

  def env_obs(self, kind, qp, info_contact, act, obs_size, obs_flags=0, coef=None):
    qp = self._a(qp)
    B = qp.shape[0]
    ic = self._a(info_contact)
    act = self._a(act).reshape(B, -1)
    self._width(act)
    obs = np.empty((B, obs_size), self.dtype)
    keep, cp = self._coef(coef)
    rc = self._fn('oracle_env_obs')(C.byref(self.cdesc), C.c_int(ENV_KIND[kind] | obs_flags << 8),
                                    C.c_int64(B), _p(qp), _p(ic), _p(act), _p(obs),
                                    C.c_int(obs_size), cp)
    del keep
    if rc:
      raise ValueError('obs size mismatch')
    return obs

  def set_act_map(self, act_map):
    """Grasp's per-action (min, range) map, (2, A)."""
    m = np.ascontiguousarray(np.asarray(act_map, np.float64))
    self._fn('oracle_set_act_map')(m.ctypes.data_as(C.POINTER(C.c_double)), C.c_int(m.shape[1]))

  def env_step(self, kind, qp, act, obs_size, n_metrics, done=None, obs_flags=0, coef=None):
    """obs_flags: BX_OBS_XY for exclude_current_positions_from_observation=False."""
    qp = self._a(qp)
    B = qp.shape[0]
    act = self._a(act).reshape(B, -1)
    self._width(act)
    out = np.empty_like(qp)
    obs = np.empty((B, obs_size), self.dtype)
    rew = np.empty(B, self.dtype)
    dn = self._a(np.zeros(B) if done is None else done).copy()
    met = np.zeros((B, n_metrics), self.dtype)
    keep, cp = self._coef(coef)
    rc = self._fn('oracle_env_step')(C.byref(self.cdesc), C.c_int(ENV_KIND[kind] | obs_flags << 8),
                                     C.c_int64(B), _p(qp), _p(act), _p(out), _p(obs),
                                     C.c_int(obs_size), _p(rew), _p(dn), _p(met),
                                     C.c_int(n_metrics), cp)
    del keep
    if rc:
      raise ValueError('obs size mismatch')
    return out, obs, rew, dn, met

  def phase(self, which, qp, aux=None):
    """0 kinetic, 1 update(acc) with aux (B,N,6) dp, 2 velocity_projection with
    aux = previous state (B,N,13)."""
    qp = self._a(qp)
    B = qp.shape[0]
    out = np.empty_like(qp)
    aux = None if aux is None else self._a(aux)
    self._fn('oracle_phase')(C.byref(self.cdesc), C.c_int(which), C.c_int64(B), _p(qp),
                             _p(aux), _p(out))
    return out

  def capsule_plane(self, qp):
    qp = self._a(qp)
    B = qp.shape[0]
    out = np.zeros((B, self.R, 10), self.dtype)
    self._fn('oracle_phase_capsule_plane')(C.byref(self.cdesc), C.c_int64(B), _p(qp), _p(out))
    return out

  def closest_segments(self, segs):
    segs = self._a(segs).reshape(-1, 4, 3)
    n = segs.shape[0]
    a = np.empty((n, 3), self.dtype)
    b = np.empty((n, 3), self.dtype)
    self._fn('oracle_closest_segments')(C.c_int64(n), _p(segs), _p(a), _p(b))
    return a, b

  def default_qp(self, angles, vels):
    assert self.creset is not None
    angles = self._a(angles)
    vels = self._a(vels)
    B = angles.shape[0]
    out = np.empty((B, self.N, 13), self.dtype)
    self._fn('oracle_default_qp')(C.byref(self.cdesc), C.byref(self.creset),
                                  C.c_int64(B), _p(angles), _p(vels), _p(out))
    return out
