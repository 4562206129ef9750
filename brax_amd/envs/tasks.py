"""Reacher, ReacherAngle, Swimmer and Pusher on MI355X: kernel env programs
BX_ENV_REACHER / REACHERANGLE / SWIMMER / PUSHER (`include/brax_amd.h`).

* Reacher (`reacher.py:172-236`): obs = [cos(angles), sin(angles), target
  xy, arm-tip vel xy, tip - target]; reward = -|tip - target| - |a|^2.
* ReacherAngle (`reacherangle.py:60-106`): the same observation; the [-1, 1]
  action is mapped onto the joints' angle limits for its Angle actuators
  before the physics (inside the step kernel); reward = -|tip - target|.
* Swimmer (`swimmer.py:153-283`): the viscous drag of the three segments is
  computed from the state inside the step kernel and appended to the action
  for the Thrusters; reward from the segments' centre of mass.
* Pusher (`pusher.py:170-242`): rewards from the state before the step.

Resets: the reachers draw joint noise and a target in a disc, the pusher
places its object in a disc and fixes goal and table, the target envs place
their target on a ring and start their per-env streams: all inside
`bx_env_reset` (the reset kernel's per-kind programs), one C call. The draws
come from the device counter RNG keyed by the reset key (JAX threefry parity
unpinned); the reset itself is pinned through `reset_from`.
"""
import ctypes as C
import math

import numpy as np
import torch

from brax_amd import _native
from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv, State, key_to_seed
from brax_amd.system import _stream


def _uniform(shape, seed, offset, lo, hi, device):
  out = torch.empty(shape, dtype=torch.float32, device=device)
  if out.numel():
    _native.check(_native.lib().bx_uniform(C.c_void_p(out.data_ptr()), out.numel(), seed,
                                           offset, float(lo), float(hi), _stream(out.device.index)))
  return out


def _slab(rng, batch_size, offset, width, lo, hi, device):
  """The (B, W) draws U(seed, g * W + k, lo, hi) of global envs g = offset..
  offset + B - 1, exactly as bx_env_reset's reset kernel draws them."""
  seed = key_to_seed(rng)
  return _uniform((batch_size, width), seed, offset * width, lo, hi, device)


# ---------------------------------------------------------------- constants
# bx_env_params.coef of each program, from the config and its body index (no
# device needed: the oracle tests build them on the CPU)

def reacher_coef(config, body_index, angle=False):
  c = np.zeros(8, np.float64)
  c[0], c[1] = body_index['target'], body_index['body1']
  if angle:
    # reacherangle.py:67-75: per action, the limit it maps [-1, 1] onto
    lim = [(l.min, l.max) for j in config.joints for l in j.angle_limit]
    if len(lim) > 2:
      raise ValueError('ReacherAngle program maps at most 2 actions')
    for i, (lo, hi) in enumerate(lim):
      c[2 + i] = lo
      c[4 + i] = hi - lo
  return c


def swimmer_coef(forward_reward_weight=1.0, ctrl_cost_weight=1e-4):
  """swimmer.py:166-193: drag constants of the mujoco swimmer."""
  viscosity, density = 0.1, 10.0
  i0, i1, i2 = 0.17278759594743870, 3.5709436495803999, 3.5709436495803999
  body_mass = 34.557519189487735
  inertia = np.array([i1 + i2 - i0, i0 + i1 - i2, i0 + i2 - i1])
  inertia = np.sqrt(inertia / (body_mass * 6))
  spherical = -3 * math.pi * np.mean(inertia) * viscosity
  fix = 0.5 * density * np.array([inertia[1] * inertia[2], inertia[0] * inertia[2],
                                  inertia[0] * inertia[1]])
  return np.array([forward_reward_weight, ctrl_cost_weight, spherical, fix[0], fix[1], fix[2],
                   0, 0], np.float64)


def pusher_coef(body_index):
  """Tip, object, goal (the step program) and table (the reset program)."""
  c = np.zeros(8, np.float64)
  c[0] = body_index['r_wrist_roll_link']
  c[1] = body_index['object']
  c[2] = body_index['goal']
  c[3] = body_index['table']
  return c


# ---------------------------------------------------------------- envs
class _KernelTask(PhysicsEnv):
  config = spring_config = None

  def __init__(self, legacy_spring=False, **kwargs):
    if legacy_spring and self.spring_config is None:
      raise NotImplementedError(f'{type(self).__name__} has no legacy_spring configuration')
    super().__init__(self.spring_config if legacy_spring else self.config, **kwargs)

  def _state(self, qp):
    """A reset State of qp: kernel observation, zero reward / done / metrics."""
    B = qp.pos.shape[0]
    dev = self.sys.device
    obs = self.observe(qp, torch.zeros((B, self.action_size), dtype=torch.float32, device=dev))
    z = torch.zeros((B,), dtype=torch.float32, device=dev)
    metrics = {k: torch.zeros_like(z) for k in self.metric_keys}
    return State(qp=qp, obs=obs, reward=z, done=torch.zeros_like(z), metrics=metrics, info={})


class Reacher(_KernelTask):
  """Trains a two-link arm's tip to a random target (`brax/envs/reacher.py`)."""
  kind = 10  # BX_ENV_REACHER
  config = robots.REACHER_CONFIG
  spring_config = robots.REACHER_SPRING_CONFIG
  metric_keys = ('reward_ctrl', 'reward_dist')  # sorted (reacher.py:180-183)
  target_sqrt = False  # ReacherAngle: dist = .2 * sqrt(u)

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    self._target_idx = self.sys.body.index['target']
    self.coef = reacher_coef(self.sys.config, self.sys.body.index,
                             angle=self.kind == 11)
    self._set_sizes()

  def reset_draws(self, rng, batch_size, env_offset=None):
    """The `reset_from` arguments `reset_batch(rng, batch_size)` builds on
    the device (reacher.py:157-165, reacherangle.py:45-50, _random_target):
    the same counter draws (W = 2D + 2 per env), the target formed on the
    host."""
    B, D, dev = int(batch_size), self.sys.num_joint_dof, self.sys.device
    off = self.env_offset if env_offset is None else int(env_offset)
    W = 2 * D + 2
    qpos = self.sys.default_angle().reshape(1, -1) + _slab(rng, B, off, W, -.1, .1, dev)[:, :D]
    qvel = _slab(rng, B, off, W, -.005, .005, dev)[:, D:2 * D]
    u = _slab(rng, B, off, W, 0., 1., dev)[:, 2 * D:].double()
    dist = .2 * (torch.sqrt(u[:, 0]) if self.target_sqrt else u[:, 0])
    ang = math.pi * 2. * u[:, 1]
    target = torch.stack([dist * torch.cos(ang), dist * torch.sin(ang),
                          torch.full_like(dist, .01)], -1).float()
    return dict(joint_angle=qpos, joint_velocity=qvel, target=target)

  def reset_from(self, joint_angle, joint_velocity, target=None):
    qp = self.sys.default_qp(joint_angle=joint_angle, joint_velocity=joint_velocity)
    if target is not None:
      qp.pos[:, self._target_idx] = torch.as_tensor(target, dtype=torch.float32,
                                                    device=self.sys.device)
    return self._state(qp)


class ReacherAngle(Reacher):
  """`brax/envs/reacherangle.py`: Angle actuators driven by [-1, 1] actions
  mapped onto the joint limits."""
  kind = 11  # BX_ENV_REACHERANGLE
  config = robots.REACHERANGLE_CONFIG
  spring_config = robots.REACHERANGLE_SPRING_CONFIG
  metric_keys = ('rewardCtrl', 'rewardDist')
  target_sqrt = True


class Swimmer(_KernelTask):
  """A three-segment swimmer in a viscous fluid (`brax/envs/swimmer.py`)."""
  kind = 12  # BX_ENV_SWIMMER
  config = robots.SWIMMER_CONFIG
  spring_config = robots.SWIMMER_SPRING_CONFIG
  # sorted (swimmer.py:204-213)
  metric_keys = ('distance_from_origin', 'forward_reward', 'reward_ctrl', 'reward_fwd',
                 'x_position', 'x_velocity', 'y_position', 'y_velocity')

  def __init__(self, forward_reward_weight=1.0, ctrl_cost_weight=1e-4, reset_noise_scale=0.1,
               exclude_current_positions_from_observation=True, legacy_reward=False, **kwargs):
    # legacy_reward is accepted and unused, as in the reference (swimmer.py:158)
    del legacy_reward
    super().__init__(**kwargs)
    self.reset_noise_scale = reset_noise_scale
    self.coef = swimmer_coef(forward_reward_weight, ctrl_cost_weight)
    from brax_amd import abi
    self.obs_flags = 0 if exclude_current_positions_from_observation else abi.OBS_XY
    self._set_sizes()

  @property
  def action_size(self):
    return 2


class Pusher(_KernelTask):
  """A 7-dof arm pushing an object to a goal (`brax/envs/pusher.py`)."""
  kind = 13  # BX_ENV_PUSHER
  config = robots.PUSHER_CONFIG
  metric_keys = ('reward_ctrl', 'reward_dist', 'reward_near')  # sorted (pusher.py:206)

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    idx = self.sys.body.index
    self._object_idx, self._goal_idx, self._table_idx = idx['object'], idx['goal'], idx['table']
    self.coef = pusher_coef(idx)
    self._set_sizes()

  def reset_draws(self, rng, batch_size, env_offset=None):
    """`reset_from` arguments of `reset_batch` (pusher.py:181-195): W = D - 2
    draws per env, qvel on the first D - 4 dofs, the object's two."""
    B, D, dev = int(batch_size), self.sys.num_joint_dof, self.sys.device
    off = self.env_offset if env_offset is None else int(env_offset)
    W = D - 2
    qvel = torch.zeros((B, D), device=dev)
    qvel[:, :D - 4] = _slab(rng, B, off, W, -.005, .005, dev)[:, :D - 4]
    x = _slab(rng, B, off, W, -.3, 0., dev)[:, D - 4].double()
    y = _slab(rng, B, off, W, -.2, .2, dev)[:, D - 3].double()
    norm = torch.sqrt(x * x + y * y)
    sc = torch.where(norm > .17, .17 / norm, torch.ones_like(norm))
    obj = torch.stack([sc * x, sc * y, torch.full_like(x, .05)], -1).float()
    qpos = self.sys.default_angle().reshape(1, -1).expand(B, -1)
    return dict(joint_angle=qpos, joint_velocity=qvel, object_pos=obj)

  def reset_from(self, joint_angle, joint_velocity, object_pos=None):
    """Reset state from explicit joint angles / velocities and the object's
    position (pusher.py:196-201: goal and table placed as the reference)."""
    qp = self.sys.default_qp(joint_angle=joint_angle, joint_velocity=joint_velocity)
    dev = self.sys.device
    qp.pos[:, self._goal_idx] = torch.tensor([0.45, 0.05, 0.05], device=dev)
    if object_pos is not None:
      qp.pos[:, self._object_idx] = torch.as_tensor(object_pos, dtype=torch.float32, device=dev)
    qp.pos[:, self._table_idx] = 0.
    return self._state(qp)


def target_coef(body_index, torso, radius, distance, height):
  """UR5E / FETCH constants: torso body, target body, the target ring."""
  c = np.zeros(8, np.float64)
  c[0], c[1] = body_index[torso], body_index['Target']
  c[2], c[3], c[4] = radius, distance, height
  return c


def rng_streams(seed, offset, batch_size, device):
  """Per-env random streams (uint32 as int32): a hash of (reset seed, global
  env id), advanced by one each env step inside the step kernel."""
  ids = torch.arange(offset, offset + batch_size, dtype=torch.int64, device=device)
  z = ids * 0x9E3779B97F4A7C15 + (int(seed) & 0x7FFFFFFFFFFFFFFF)
  z = (z ^ (z >> 31)) * 0x94D049BB133111EB
  return (z ^ (z >> 29)).to(torch.int32)


class Ur5e(_KernelTask):
  """A UR5e arm reaching for targets (`brax/envs/ur5e.py`): egocentric
  observation in the wrist's frame; a hit target is teleported to a fresh
  spot (the env's device stream; JAX key parity unpinned)."""
  kind = 14  # BX_ENV_UR5E
  config = robots.UR5E_CONFIG
  spring_config = robots.UR5E_SPRING_CONFIG
  metric_keys = ('hits', 'movingToTarget', 'weightedHits')  # sorted (ur5e.py:64-68)
  torso = 'wrist_3_link'
  needs_rng = True  # the step reads and advances info['rng']
  ring = (.02, .5, .5)  # target radius, distance, height (ur5e.py:51-54,126-135)

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    self.target_idx = self.sys.body.index['Target']
    self.coef = target_coef(self.sys.body.index, self.torso, *self.ring)
    self._set_sizes()

  def reset_draws(self, rng, batch_size, env_offset=None):
    """`reset_from` arguments of `reset_batch` (ur5e.py:41-46,117-125): the
    default pose at rest, the target's two draws per env on the ring."""
    B, D, dev = int(batch_size), self.sys.num_joint_dof, self.sys.device
    off = self.env_offset if env_offset is None else int(env_offset)
    u = _slab(rng, B, off, 2, 0., 1., dev).double()
    radius, distance, height = self.ring
    dist = radius + distance * u[:, 0]
    ang = math.pi * 2. * u[:, 1]
    target = torch.stack([dist * torch.cos(ang), dist * torch.sin(ang),
                          torch.full_like(dist, height)], -1).float()
    return dict(joint_angle=self.sys.default_angle().reshape(1, -1).expand(B, -1),
                joint_velocity=torch.zeros((B, D), device=dev), target=target)

  def reset_from(self, joint_angle, joint_velocity, target=None):
    qp = self.sys.default_qp(joint_angle=joint_angle, joint_velocity=joint_velocity)
    if target is not None:
      qp.pos[:, self.target_idx] = torch.as_tensor(target, dtype=torch.float32,
                                                   device=self.sys.device)
    st = self._state(qp)
    st.info['rng'] = rng_streams(0, self.env_offset, qp.pos.shape[0], self.sys.device)
    return st


class Fetch(Ur5e):
  """A dog of boxes fetching targets (`brax/envs/fetch.py`): Ur5e's
  egocentric observation around the Torso, plus upright / height / facing
  rewards."""
  kind = 15  # BX_ENV_FETCH
  config = robots.FETCH_CONFIG
  spring_config = robots.FETCH_SPRING_CONFIG
  # sorted (fetch.py:47-53)
  metric_keys = ('hits', 'movingToTarget', 'torsoHeight', 'torsoIsUp', 'weightedHits')
  torso = 'Torso'
  ring = (2., 15., 1.)  # fetch.py:36-39,124-134


def grasp_coef(body_index):
  """GRASP constants: palm, object, target, hand bodies and the target ring
  (grasp.py:35-41)."""
  c = np.zeros(8, np.float64)
  c[0], c[1] = body_index['HandPalm'], body_index['Object']
  c[2], c[3] = body_index['Target'], body_index['HandThumbProximal']
  c[4], c[5], c[6] = 1.1, 10., 8.
  return c


def grasp_act_map(config):
  """grasp.py:42-52: per action (min, range), the joints' angle limits then
  the palm's translation range; (2, A)."""
  lim = [(l.min, l.max) for j in config.joints for l in j.angle_limit]
  lo = [l[0] for l in lim] + [-10., -10., 3.5]
  rg = [l[1] - l[0] for l in lim] + [20., 20., 10.]
  return np.array([lo, rg], np.float64)


class Grasp(_KernelTask):
  """A hand grasping an object and carrying it to targets
  (`brax/envs/grasp.py`): [-1, 1] actions mapped onto the joints' angle
  limits plus 3 that move the palm before the physics (inside the step
  kernel); observation in the palm's frame; a hit target is teleported (the
  env's device stream; JAX key parity unpinned)."""
  kind = 16  # BX_ENV_GRASP
  config = robots.GRASP_CONFIG
  spring_config = robots.GRASP_SPRING_CONFIG
  # sorted (grasp.py:47-53)
  metric_keys = ('closeToObject', 'hits', 'movingObjectToTarget', 'movingToObject',
                 'touchingObject')
  needs_rng = True

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    self.target_idx = self.sys.body.index['Target']
    self.coef = grasp_coef(self.sys.body.index)
    self.act_map = torch.as_tensor(grasp_act_map(self.sys.config), dtype=torch.float32,
                                   device=self.sys.device).contiguous()
    self._set_sizes()

  @property
  def action_size(self):
    return self.sys.num_joint_dof + self.sys.num_forces_dof + 3  # grasp.py:128-130

  def _params(self, opts=None, first_qp=None, first_obs=None):
    p = super()._params(opts, first_qp, first_obs)
    p.act_map = self.act_map.data_ptr() if hasattr(self, 'act_map') else None
    return p

  def reset_from(self, joint_angle, joint_velocity):
    qp = self.sys.default_qp(joint_angle=joint_angle, joint_velocity=joint_velocity)
    st = self._state(qp)
    st.info['rng'] = rng_streams(0, self.env_offset, qp.pos.shape[0], self.sys.device)
    return st
