"""ctypes mirror of `include/brax_amd.h` (structs only, no library loading).

`make_desc` / `make_reset_desc` turn the compiler's numpy descriptor into the
C structs; the returned keep-alive list must outlive every call that reads the
struct (create copies it to the device, so only the create call needs it).
"""
import ctypes as C

import numpy as np

i32p = C.POINTER(C.c_int32)
f64p = C.POINTER(C.c_double)
f32p = C.POINTER(C.c_float)

ABI_VERSION = 13  # include/brax_amd.h BX_ABI_VERSION

_DESC_FIELDS = [
    ('n_bodies', C.c_int32), ('n_joints', C.c_int32), ('n_actuators', C.c_int32),
    ('n_rows', C.c_int32), ('n_groups', C.c_int32),
    ('substeps', C.c_int32), ('action_size', C.c_int32), ('num_joint_dof', C.c_int32),
    ('dt', C.c_double), ('h', C.c_double), ('gravity', C.c_double * 3),
    ('velocity_damping', C.c_double), ('angular_damping', C.c_double),
    ('body_mass', f64p), ('body_inv_inertia', f64p), ('pos_mask', f64p),
    ('rot_mask', f64p), ('quat_mask', f64p),
    ('joint_type', i32p), ('joint_dof', i32p), ('joint_free_dofs', i32p),
    ('joint_body_p', i32p), ('joint_body_c', i32p), ('joint_group', i32p),
    ('joint_off_p', f64p), ('joint_off_c', f64p), ('joint_axis_p', f64p),
    ('joint_axis_c', f64p), ('joint_limit', f64p), ('joint_damping', f64p),
    ('joint_scale_pos', f64p), ('joint_scale_ang', f64p),
    ('act_type', i32p), ('act_joint', i32p), ('act_index', i32p),
    ('act_group', i32p), ('act_strength', f64p),
    ('col_oneway', i32p), ('col_fn', i32p), ('col_scale', f64p),
    ('col_velocity_threshold', f64p), ('col_baumgarte_erp', f64p),
    ('row_group', i32p), ('row_body_a', i32p), ('row_body_b', i32p),
    ('row_a_pos', f64p), ('row_a_end', f64p), ('row_a_radius', f64p),
    ('row_b_pos', f64p), ('row_b_end', f64p), ('row_b_radius', f64p),
    ('row_friction', f64p), ('row_elasticity', f64p),
    ('n_forces', C.c_int32), ('force_type', i32p), ('force_body', i32p),
    ('force_index', i32p), ('force_strength', f64p),
    ('col_cutoff', i32p), ('row_flat', i32p),
    ('dynamics_mode', C.c_int32), ('joint_stiffness', f64p),
    ('joint_spring_damping', f64p), ('joint_limit_strength', f64p),
    ('row_ext', f64p), ('row_hm', i32p), ('n_hm', C.c_int32), ('hm_data', f64p),
    ('n_hull', C.c_int32), ('hull_vert', f64p), ('hull_face', f64p), ('hull_norm', f64p),
    ('row_nn_masked', i32p),
]

DYN_PBD, DYN_LEGACY_SPRING = 0, 1
OBS_XY = 1  # BX_OBS_XY: exclude_current_positions_from_observation=False
_SPRING_FIELDS = ('joint_stiffness', 'joint_spring_damping', 'joint_limit_strength')


class BxDesc(C.Structure):
  _fields_ = _DESC_FIELDS


class BxResetDesc(C.Structure):
  _fields_ = [
      ('n_fk', C.c_int32), ('fk_body_p', i32p), ('fk_body_c', i32p),
      ('fk_dof_index', i32p), ('fk_rot', f64p), ('fk_ref', f64p),
      ('fk_off_p', f64p), ('fk_off_c', f64p), ('base_qp', f64p),
      ('n_zpts', C.c_int32), ('zpt_body', i32p), ('zpt_local', f64p),
      ('zpt_radius', f64p), ('body_zero_cand', i32p), ('body_root_group', i32p),
      ('n_root_groups', C.c_int32), ('default_angle', f64p),
  ]


class BxField(C.Structure):
  _fields_ = [('ptr', C.c_void_p), ('env_stride', C.c_int64),
              ('body_stride', C.c_int64)]


class BxQP(C.Structure):
  _fields_ = [('pos', BxField), ('rot', BxField), ('vel', BxField),
              ('ang', BxField)]


class BxInfo(C.Structure):
  _fields_ = [('contact_vel', BxField), ('contact_ang', BxField),
              ('actuator_vel', BxField), ('actuator_ang', BxField),
              ('contact_pos', C.c_void_p), ('contact_normal', C.c_void_p),
              ('contact_penetration', C.c_void_p),
              ('joint_vel', BxField), ('joint_ang', BxField),
              ('contact_cell', C.c_void_p)]


class BxEnvState(C.Structure):
  _fields_ = [('qp', BxQP), ('obs', C.c_void_p), ('reward', C.c_void_p),
              ('done', C.c_void_p), ('metrics', C.c_void_p),
              ('steps', C.c_void_p), ('truncation', C.c_void_p), ('rng', C.c_void_p)]


class BxEnvParams(C.Structure):
  _fields_ = [('kind', C.c_int32), ('obs_size', C.c_int32),
              ('n_metrics', C.c_int32), ('episode_length', C.c_int32),
              ('action_repeat', C.c_int32), ('auto_reset', C.c_int32),
              ('obs_flags', C.c_int32), ('coef', C.c_float * 8),
              ('first_qp', BxQP), ('first_obs', C.c_void_p), ('act_map', C.c_void_p)]


def _arr(x, dtype):
  a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
  if a.size == 0:
    a = np.zeros(1, dtype)
  return a


def make_desc(d):
  """numpy descriptor dict -> (BxDesc, keepalive)."""
  keep = []
  s = BxDesc()
  s.n_bodies = int(d['n_bodies'])
  s.n_joints = len(d['joint_type'])
  s.n_actuators = len(d['act_type'])
  s.n_rows = len(d['row_group'])
  s.n_groups = len(d['col_oneway'])
  s.n_forces = len(d.get('force_type', ()))
  s.substeps = int(d['substeps'])
  s.action_size = int(d.get('action_size', 0))
  s.num_joint_dof = int(d.get('num_joint_dof', 0))
  s.dt = float(d['dt'])
  s.h = float(d['h'])
  for k in range(3):
    s.gravity[k] = float(d['gravity'][k])
  s.velocity_damping = float(d['velocity_damping'])
  s.angular_damping = float(d['angular_damping'])
  s.dynamics_mode = int(d.get('dynamics_mode', DYN_PBD))
  s.n_hm = len(d.get('hm_data', ()))
  s.n_hull = len(d.get('hull_vert', ()))
  for name, ctype in _DESC_FIELDS:
    if ctype is i32p or ctype is f64p:
      if name in d:
        v = d[name]
      elif name == 'col_cutoff':
        v = np.zeros(len(d['col_oneway']))
      elif name == 'row_flat':
        v = -np.ones(len(d['row_group']))
      elif name == 'row_nn_masked':
        v = np.zeros(len(d['row_group']))
      elif name.startswith('force_'):
        v = np.zeros(0)
      elif name in _SPRING_FIELDS:
        v = np.zeros(len(d['joint_type']))
      elif name == 'row_ext':
        v = np.zeros((len(d['row_group']), 16))
      elif name == 'row_hm':
        v = np.tile([-1, 0], (len(d['row_group']), 1))
      elif name in ('hm_data', 'hull_vert', 'hull_face', 'hull_norm'):
        v = np.zeros(0)
      else:
        raise KeyError(name)
      a = _arr(v, np.int32 if ctype is i32p else np.float64)
      keep.append(a)
      setattr(s, name, a.ctypes.data_as(ctype))
  return s, keep


def info_rows(d):
  """Contact rows of `Info` (`_get_contact_info`, system.py:36-43): every row
  of a Pairs group, `cutoff` rows of a NearNeighbors group."""
  groups = np.asarray(d['row_group'])
  cut = np.asarray(d.get('col_cutoff', np.zeros(len(d['col_oneway']))))
  return int(sum(int(c) if c else int((groups == g).sum()) for g, c in enumerate(cut)))


def make_reset_desc(r, num_joint_dof=None):
  """Reset descriptor -> (BxResetDesc, keepalive). default_angle is padded
  with zeros to num_joint_dof (the kernels' joint-angle stride)."""
  keep = []
  r = dict(r)
  da = np.asarray(r.get('default_angle', np.zeros(0)), np.float64)
  n = len(da) if num_joint_dof is None else int(num_joint_dof)
  r['default_angle'] = np.pad(da, (0, max(n - len(da), 0)))[:max(n, len(da))]
  s = BxResetDesc()
  s.n_fk = len(r['fk_body_p'])
  s.n_zpts = len(r['zpt_body'])
  s.n_root_groups = int(r['n_root_groups'])
  for name, ctype in BxResetDesc._fields_:
    if ctype is i32p or ctype is f64p:
      a = _arr(r[name], np.int32 if ctype is i32p else np.float64)
      keep.append(a)
      setattr(s, name, a.ctypes.data_as(ctype))
  return s, keep
