"""The other registered envs: physics on the fused HIP step, env layer in torch.

`TorchEnv.step` is one `System.step` kernel launch (`bx_system_step`) plus the
env's observation / reward / done as device tensor ops, batched over the
leading env axis. The systems are the reference envs' pbd configs
(`brax_amd/envs/robots.py`); the env code follows the reference modules
cited per class. Episode / AutoReset wrappers run as device tensor ops above
these envs (`wrappers.py`), with the reference's semantics.

Reset noise and random targets come from the device counter RNG keyed by the
reset key (`bx_uniform`); JAX threefry parity is unpinned, so
parity is defined on explicit states (`reset_from`).
"""
import ctypes as C

import torch

from brax_amd import _native
from brax_amd import math as bm
from brax_amd.base import QP
from brax_amd.envs import robots
from brax_amd.envs.env import Env, State, key_to_seed
from brax_amd.system import _stream


def _uniform(shape, seed, offset, lo, hi, device):
  out = torch.empty(shape, dtype=torch.float32, device=device)
  if out.numel():
    _native.check(_native.lib().bx_uniform(C.c_void_p(out.data_ptr()), out.numel(), seed,
                                           offset, float(lo), float(hi), _stream()))
  return out


def _zeros(B, device):
  return torch.zeros((B,), dtype=torch.float32, device=device)


class TorchEnv(Env):
  """An env whose physics is the fused step kernel and whose env layer is
  torch (`env.py:39-71` API). States are batched: leaves have a leading
  (B,) axis."""

  config = None          # robot description text
  qpos_noise = (0., 0.)  # reset joint-angle noise range
  qvel_noise = (0., 0.)  # reset joint-velocity noise range
  metric_keys = ()

  def __init__(self, batch_size=None, device=None, legacy_spring=False, **kwargs):
    if legacy_spring:
      raise NotImplementedError('legacy_spring dynamics are outside the MI355X path')
    super().__init__(self.config, device=device)
    self.batch_size = batch_size
    self.dev = self.sys.device

  @property
  def observation_size(self):
    return self.obs_size

  # ---------------------------------------------------------------- reset
  def reset(self, rng) -> State:
    return self.reset_batch(rng, self.batch_size or 1)

  def reset_batch(self, rng, batch_size):
    seed = key_to_seed(rng)
    D = self.sys.num_joint_dof
    qpos = self.sys.default_angle().reshape(1, -1) + _uniform(
        (batch_size, D), seed, 0, *self.qpos_noise, self.dev)
    qvel = _uniform((batch_size, D), seed, batch_size * D, *self.qvel_noise, self.dev)
    extra = self._reset_extra(seed, batch_size)
    return self.reset_from(qpos, qvel, **extra)

  def _reset_extra(self, seed, batch_size):  # pylint: disable=unused-argument
    return {}

  def reset_from(self, joint_angle, joint_velocity, **extra) -> State:
    """Reset state from explicit joint angles / velocities (B, num_joint_dof)."""
    qp = self.sys.default_qp(joint_angle=joint_angle, joint_velocity=joint_velocity)
    qp = self._reset_qp(qp, **extra)
    B = qp.pos.shape[0]
    obs = self._get_obs(qp, None)
    z = _zeros(B, self.dev)
    metrics = {k: torch.zeros_like(z) for k in self.metric_keys}
    return State(qp=qp, obs=obs, reward=z, done=torch.zeros_like(z), metrics=metrics,
                 info=self._reset_info(**extra))

  def _reset_qp(self, qp, **extra):  # pylint: disable=unused-argument
    return qp

  def _reset_info(self, **extra):  # pylint: disable=unused-argument
    return {}

  # ---------------------------------------------------------------- step
  def _action(self, action, B):
    a = torch.as_tensor(action, dtype=torch.float32, device=self.dev)
    if a.dim() == 1:
      a = a.reshape(1, -1).expand(B, -1)
    return a

  def step(self, state: State, action) -> State:
    B = state.qp.pos.shape[0]
    action = self._action(action, B)
    qp, info = self.sys.step(state.qp, self._system_action(state, action))
    return self._step(state, action, qp, info)

  def _system_action(self, state, action):  # pylint: disable=unused-argument
    return action

  def _get_obs(self, qp, info):
    raise NotImplementedError

  def _step(self, state, action, qp, info):
    raise NotImplementedError


def _replace_metrics(state, **kw):
  m = dict(state.metrics)
  m.update(kw)
  return m


class _Locomotion2D(TorchEnv):
  """Hopper / Walker2d (`hopper.py:120-250`, `walker2d.py:130-253`)."""

  metric_keys = ('reward_forward', 'reward_ctrl', 'reward_healthy', 'x_position', 'x_velocity')

  def __init__(self, forward_reward_weight=1.0, ctrl_cost_weight=1e-3, healthy_reward=1.0,
               terminate_when_unhealthy=True, healthy_z_range=(0.7, float('inf')),
               healthy_angle_range=(-0.2, 0.2), reset_noise_scale=5e-3,
               exclude_current_positions_from_observation=True, **kwargs):
    super().__init__(**kwargs)
    self._fw, self._cw, self._hr = forward_reward_weight, ctrl_cost_weight, healthy_reward
    self._term = terminate_when_unhealthy
    self._z, self._ang = healthy_z_range, healthy_angle_range
    self.qpos_noise = self.qvel_noise = (-reset_noise_scale, reset_noise_scale)
    self._exclude = exclude_current_positions_from_observation
    D = self.sys.joints[0]._hi - self.sys.joints[0]._lo  # pylint: disable=protected-access
    self.obs_size = (1 if self._exclude else 2) + 1 + D + 2 + 1 + D

  def _get_obs(self, qp, info):
    ja, jv = self.sys.joints[0].angle_vel(qp)
    ang_y = bm.quat_to_euler(qp.rot[:, 0])[:, 1:2]
    pos = qp.pos[:, 0, 2:] if self._exclude else qp.pos[:, 0][:, [0, 2]]
    qvel = [qp.vel[:, 0][:, [0, 2]], qp.ang[:, 0, 1:2], jv]
    return torch.cat([pos, ang_y, ja] + qvel, -1)

  def _step(self, state, action, qp, info):
    dt = float(self.sys.config.dt)
    x_velocity = (qp.pos[:, 0, 0] - state.qp.pos[:, 0, 0]) / dt
    forward_reward = self._fw * x_velocity
    ang_y = bm.quat_to_euler(qp.rot[:, 0])[:, 1]
    z = qp.pos[:, 0, 2]
    one, zero = torch.ones_like(z), torch.zeros_like(z)
    healthy = torch.where(z < self._z[0], zero, one)
    healthy = torch.where(z > self._z[1], zero, healthy)
    healthy = torch.where(ang_y > self._ang[1], zero, healthy)
    healthy = torch.where(ang_y < self._ang[0], zero, healthy)
    healthy_reward = self._hr * one if self._term else self._hr * healthy
    ctrl_cost = self._cw * (action * action).sum(-1)
    obs = self._get_obs(qp, info)
    reward = forward_reward + healthy_reward - ctrl_cost
    done = 1.0 - healthy if self._term else zero
    metrics = _replace_metrics(state, reward_forward=forward_reward, reward_ctrl=-ctrl_cost,
                               reward_healthy=healthy_reward, x_position=qp.pos[:, 0, 0],
                               x_velocity=x_velocity)
    return state.replace(qp=qp, obs=obs, reward=reward, done=done, metrics=metrics)


class Hopper(_Locomotion2D):
  """`brax/envs/hopper.py`."""
  config = robots.HOPPER_CONFIG


class Walker2d(_Locomotion2D):
  """`brax/envs/walker2d.py` (its own healthy ranges, walker2d.py:132-141)."""
  config = robots.WALKER2D_CONFIG

  def __init__(self, healthy_z_range=(0.7, 2.0), healthy_angle_range=(-1.0, 1.0), **kwargs):
    super().__init__(healthy_z_range=healthy_z_range, healthy_angle_range=healthy_angle_range,
                     **kwargs)


class InvertedPendulum(TorchEnv):
  """`brax/envs/inverted_pendulum.py:124-166`; action_size 1 (the thruster's
  three indices clip to action[0])."""
  config = robots.INVERTED_PENDULUM_CONFIG
  qpos_noise = qvel_noise = (-0.01, 0.01)
  obs_size = 4

  @property
  def action_size(self):
    return 1

  def _get_obs(self, qp, info):
    ja, jv = self.sys.joints[0].angle_vel(qp)
    return torch.cat([qp.pos[:, 0, :1], ja, qp.vel[:, 0, :1], jv], -1)

  def _step(self, state, action, qp, info):
    obs = self._get_obs(qp, info)
    reward = torch.ones_like(obs[:, 0])
    done = torch.where(obs[:, 1].abs() > .2, 1.0, 0.0)
    return state.replace(qp=qp, obs=obs, reward=reward, done=done)


class InvertedDoublePendulum(TorchEnv):
  """`brax/envs/inverted_double_pendulum.py:131-186`."""
  config = robots.INVERTED_DOUBLE_PENDULUM_CONFIG
  qpos_noise = qvel_noise = (-0.01, 0.01)
  obs_size = 8

  @property
  def action_size(self):
    return 1

  def _get_obs(self, qp, info):
    ja, jv = self.sys.joints[0].angle_vel(qp)
    return torch.cat([qp.pos[:, 0, :1], torch.sin(ja), torch.cos(ja), qp.vel[:, 0, :1], jv], -1)

  def _step(self, state, action, qp, info):
    _, jv = self.sys.joints[0].angle_vel(qp)
    tip, _ = qp[:, 2].to_world(torch.tensor([0., 0., .3], device=self.dev))
    x, y = tip[:, 0], tip[:, 2]
    dist_penalty = 0.01 * x ** 2 + (y - 2) ** 2
    v1, v2 = jv[:, 0], jv[:, 1]
    vel_penalty = 1e-3 * v1 ** 2 + 5e-3 * v2 ** 2
    obs = self._get_obs(qp, info)
    reward = 10.0 - dist_penalty - vel_penalty
    done = torch.where(y <= 1, 1.0, 0.0)
    return state.replace(qp=qp, obs=obs, reward=reward, done=done)


class Swimmer(TorchEnv):
  """`brax/envs/swimmer.py:153-290`: viscous drag fed to the three Thrusters
  through the action tail."""
  config = robots.SWIMMER_CONFIG
  metric_keys = ('reward_fwd', 'reward_ctrl', 'x_position', 'y_position',
                 'distance_from_origin', 'x_velocity', 'y_velocity', 'forward_reward')

  def __init__(self, forward_reward_weight=1.0, ctrl_cost_weight=1e-4, reset_noise_scale=0.1,
               exclude_current_positions_from_observation=True, legacy_reward=False, **kwargs):
    if legacy_reward:
      raise NotImplementedError('legacy_reward')
    super().__init__(**kwargs)
    self._fw, self._cw = forward_reward_weight, ctrl_cost_weight
    self.qpos_noise = self.qvel_noise = (-reset_noise_scale, reset_noise_scale)
    self._exclude = exclude_current_positions_from_observation
    viscosity, density = 0.1, 10.0
    i0, i1, i2 = 0.17278759594743870, 3.5709436495803999, 3.5709436495803999
    body_mass = 34.557519189487735
    inertia = torch.tensor([i1 + i2 - i0, i0 + i1 - i2, i0 + i2 - i1], dtype=torch.float64)
    inertia = torch.sqrt(inertia / (body_mass * 6))
    self._spherical_drag = float(-3 * bm.PI * inertia.mean() * viscosity)
    self._fix_drag = (0.5 * density * torch.stack([inertia[1] * inertia[2], inertia[0] * inertia[2],
                                                   inertia[0] * inertia[1]])).float().to(self.dev)
    D = self.sys.joints[0]._hi - self.sys.joints[0]._lo  # pylint: disable=protected-access
    self.obs_size = (1 if self._exclude else 3) + D + 2 + 1 + D
    self._mass = torch.as_tensor(self.sys.body.mass[:-1], dtype=torch.float32, device=self.dev)

  @property
  def action_size(self):
    return 2

  def _viscous_force(self, qp):
    """`swimmer.py:246-255`."""
    vel, rot = qp.vel[:, :-1], qp.rot[:, :-1]
    force = vel * self._spherical_drag
    lv = bm.rotate(vel, bm.quat_inv(rot))
    # `force -= jp.diag(fix_drag * |v| * v)`: jp.diag of the (3 bodies, 3)
    # matrix is its diagonal [d00, d11, d22], broadcast over every body's row
    d = self._fix_drag * lv.abs() * lv
    force = force - d.diagonal(dim1=1, dim2=2)[:, None, :]
    force = bm.rotate(force, rot)
    return torch.clamp(force, -5., 5.)

  def _system_action(self, state, action):
    force = self._viscous_force(state.qp)
    return torch.cat([action, force.reshape(force.shape[0], -1)], -1)

  def _center_of_mass(self, qp):
    return (self._mass[None, :, None] * qp.pos[:, :-1]).sum(1) / self._mass.sum()

  def _get_obs(self, qp, info):
    ja, jv = self.sys.joints[0].angle_vel(qp)
    ang_z = bm.quat_to_euler(qp.rot[:, 0])[:, 2:3]
    qpos = [ang_z, ja] if self._exclude else [qp.pos[:, 0, :2], ang_z, ja]
    qvel = [qp.vel[:, 0, :2], qp.ang[:, 0, 2:], jv]
    return torch.cat(qpos + qvel, -1)

  def _step(self, state, action, qp, info):
    dt = float(self.sys.config.dt)
    com_before = self._center_of_mass(state.qp)
    com_after = self._center_of_mass(qp)
    velocity = (com_after - com_before) / dt
    forward_reward = self._fw * velocity[:, 0]
    ctrl_cost = self._cw * (action * action).sum(-1)
    obs = self._get_obs(qp, info)
    reward = forward_reward - ctrl_cost
    metrics = _replace_metrics(
        state, reward_fwd=forward_reward, reward_ctrl=-ctrl_cost, x_position=com_after[:, 0],
        y_position=com_after[:, 1], distance_from_origin=torch.linalg.norm(qp.pos[:, 0], dim=-1),
        x_velocity=velocity[:, 0], y_velocity=velocity[:, 1], forward_reward=forward_reward)
    return state.replace(qp=qp, obs=obs, reward=reward, metrics=metrics)


class Reacher(TorchEnv):
  """`brax/envs/reacher.py:150-236`."""
  config = robots.REACHER_CONFIG
  qpos_noise = (-.1, .1)
  qvel_noise = (-.005, .005)
  metric_keys = ('reward_dist', 'reward_ctrl')
  target_sqrt = False  # ReacherAngle draws dist = .2 * sqrt(u)

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    self._target_idx = self.sys.body.index['target']
    self._arm_idx = self.sys.body.index['body1']
    D = self.sys.joints[0]._hi - self.sys.joints[0]._lo  # pylint: disable=protected-access
    self.obs_size = 2 * D + 2 + 2 + 3

  def _reset_extra(self, seed, batch_size):
    u = _uniform((2, batch_size), seed ^ 0x7A46E7, 0, 0., 1., self.dev)
    dist = .2 * (torch.sqrt(u[0]) if self.target_sqrt else u[0])
    ang = bm.PI * 2. * u[1]
    target = torch.stack([dist * torch.cos(ang), dist * torch.sin(ang),
                          torch.full_like(dist, .01)], -1)
    return {'target': target}

  def reset_from(self, joint_angle, joint_velocity, target=None, **extra):
    return super().reset_from(joint_angle, joint_velocity, target=target, **extra)

  def _reset_qp(self, qp, target=None):
    if target is None:
      return qp
    pos = qp.pos.clone()
    pos[:, self._target_idx] = torch.as_tensor(target, dtype=torch.float32, device=self.dev)
    return QP(pos=pos, rot=qp.rot, vel=qp.vel, ang=qp.ang)

  def _get_obs(self, qp, info):
    ja, _ = self.sys.joints[0].angle_vel(qp)
    target = qp.pos[:, self._target_idx]
    tip_pos, tip_vel = qp[:, self._arm_idx].to_world(torch.tensor([0.11, 0., 0.], device=self.dev))
    return torch.cat([torch.cos(ja), torch.sin(ja), target[:, :2], tip_vel[:, :2],
                      tip_pos - target], -1)

  def _step(self, state, action, qp, info):
    obs = self._get_obs(qp, info)
    reward_dist = -torch.linalg.norm(obs[:, -3:], dim=-1)
    reward_ctrl = -(action * action).sum(-1)
    metrics = _replace_metrics(state, reward_dist=reward_dist, reward_ctrl=reward_ctrl)
    return state.replace(qp=qp, obs=obs, reward=reward_dist + reward_ctrl, metrics=metrics)


class ReacherAngle(Reacher):
  """`brax/envs/reacherangle.py:30-106`: [-1, 1] actions mapped onto the
  joints' angle limits for the Angle actuators."""
  config = robots.REACHERANGLE_CONFIG
  metric_keys = ('rewardDist', 'rewardCtrl')
  target_sqrt = True

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    lim = [(l.min, l.max) for j in self.sys.config.joints for l in j.angle_limit]
    self._min_act = torch.tensor([l[0] for l in lim], dtype=torch.float32, device=self.dev)
    self._range_act = torch.tensor([l[1] - l[0] for l in lim], dtype=torch.float32,
                                   device=self.dev)

  def _system_action(self, state, action):
    return self._min_act + self._range_act * ((action + 1) / 2.)

  def _step(self, state, action, qp, info):
    obs = self._get_obs(qp, info)
    reward_dist = -torch.linalg.norm(obs[:, -3:], dim=-1)
    metrics = {'rewardDist': reward_dist, 'rewardCtrl': torch.zeros_like(reward_dist)}
    return state.replace(qp=qp, obs=obs, reward=reward_dist, metrics=metrics)


class Acrobot(TorchEnv):
  """`brax/envs/acrobot.py:40-95`."""
  config = robots.ACROBOT_CONFIG
  qpos_noise = qvel_noise = (-.01, .01)
  metric_keys = ('dist_penalty', 'vel_penalty', 'alive_bonus', 'r_tot')
  obs_size = 4

  @property
  def action_size(self):
    return 1

  def _get_obs(self, qp, info):
    ja, jv = self.sys.joints[0].angle_vel(qp)
    return torch.cat([ja, jv], -1)

  def _step(self, state, action, qp, info):
    ja, jv = self.sys.joints[0].angle_vel(qp)
    obs = torch.cat([ja, jv], -1)
    dist_penalty = ja[:, 0] ** 2 + ja[:, 1] ** 2
    vel_penalty = 1e-3 * (jv[:, 0] ** 2 + jv[:, 1] ** 2)
    r = 10.0 - dist_penalty - vel_penalty
    metrics = _replace_metrics(state, dist_penalty=dist_penalty, vel_penalty=vel_penalty,
                               r_tot=r)
    return state.replace(qp=qp, obs=obs, reward=r, done=torch.zeros_like(r), metrics=metrics)
