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
                                           offset, float(lo), float(hi), _stream(out.device.index)))
  return out


def _zeros(B, device):
  return torch.zeros((B,), dtype=torch.float32, device=device)


class TorchEnv(Env):
  """An env whose physics is the fused step kernel and whose env layer is
  torch (`env.py:39-71` API). States are batched: leaves have a leading
  (B,) axis."""

  config = None          # robot description text
  spring_config = None   # its legacy_spring variant (`_SYSTEM_CONFIG_SPRING`)
  qpos_noise = (0., 0.)  # reset joint-angle noise range
  qvel_noise = (0., 0.)  # reset joint-velocity noise range
  metric_keys = ()

  def __init__(self, batch_size=None, device=None, legacy_spring=False, **kwargs):
    if legacy_spring and self.spring_config is None:
      raise NotImplementedError(f'{type(self).__name__} has no legacy_spring configuration')
    super().__init__(self.spring_config if legacy_spring else self.config, device=device)
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
    qp, info = self.sys.step(*self._pre_step(state, action))
    return self._step(state, action, qp, info)

  def _pre_step(self, state, action):
    """(qp, action) handed to System.step."""
    return state.qp, self._system_action(state, action)

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


def _contacts(info, n):
  """`jp.where(sum(contact.vel^2) > 1e-5, 1, 0)` per body (grasp.py:163-164)."""
  if info is None:
    return torch.zeros((1, n))
  mag = (info.contact.vel * info.contact.vel).sum(-1)
  return torch.where(mag > 0.00001, 1.0, 0.0)


class _TargetEnv(TorchEnv):
  """Shared pieces of Ur5e / Grasp: an egocentric frame, contact flags from
  Info, and a target teleported after a hit (device RNG; the reference keys
  it by the state's rng, parity unpinned)."""

  def _random_target(self, seed, B):
    raise NotImplementedError

  def reset_batch(self, rng, batch_size):
    seed = key_to_seed(rng)
    qp0 = self.sys.default_qp()
    qp = QP(*(t.unsqueeze(0).expand((batch_size,) + t.shape).contiguous()
              for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
    qp = self._reset_target(qp, seed, batch_size)
    info = self.sys.info(qp)
    obs = self._get_obs(qp, info)
    z = _zeros(batch_size, self.dev)
    metrics = {k: torch.zeros_like(z) for k in self.metric_keys}
    ctr = torch.full((batch_size,), seed & 0x7FFFFFFF, dtype=torch.float64, device=self.dev)
    return State(qp=qp, obs=obs, reward=z, done=torch.zeros_like(z), metrics=metrics,
                 info={'rng': ctr})

  def _reset_target(self, qp, seed, B):  # pylint: disable=unused-argument
    return qp

  def _teleport(self, state, qp, hit):
    """Targets that were hit move to a fresh random spot."""
    B = qp.pos.shape[0]
    seed = int(state.info['rng'][0].item()) if 'rng' in state.info else 0
    target = self._random_target(seed + 1, B)
    pos = qp.pos.clone()
    pos[:, self.target_idx] = torch.where(hit[:, None] != 0, target, qp.pos[:, self.target_idx])
    info = dict(state.info)
    info['rng'] = state.info.get('rng', torch.zeros(B, dtype=torch.float64,
                                                    device=self.dev)) + 1
    return QP(pos=pos, rot=qp.rot, vel=qp.vel, ang=qp.ang), info


class Grasp(_TargetEnv):
  """`brax/envs/grasp.py:29-190`: Angle actuators driven through [-1, 1]
  actions, plus 3 actions that translate the palm before the physics step."""
  config = robots.GRASP_CONFIG
  spring_config = robots.GRASP_SPRING_CONFIG
  metric_keys = ('hits', 'touchingObject', 'movingToObject', 'movingObjectToTarget',
                 'closeToObject')

  def __init__(self, **kwargs):
    super().__init__(**kwargs)
    idx = self.sys.body.index
    self.object_idx, self.target_idx = idx['Object'], idx['Target']
    self.hand_idx, self.palm_idx = idx['HandThumbProximal'], idx['HandPalm']
    self.target_radius, self.target_distance, self.target_height = 1.1, 10., 8.
    lim = [(l.min, l.max) for j in self.sys.config.joints for l in j.angle_limit]
    self._min_act = torch.tensor([l[0] for l in lim] + [-10, -10, 3.5], dtype=torch.float32,
                                 device=self.dev)
    self._range_act = torch.tensor([l[1] - l[0] for l in lim] + [20, 20, 10],
                                   dtype=torch.float32, device=self.dev)
    N = self.sys.num_bodies
    self.obs_size = 1 + 3 + 1 + 3 + 3 * N + 3 * N + 3 + 3 + 1 + 1 + 3 + 1 + N

  @property
  def action_size(self):
    return self.sys.num_joint_dof + self.sys.num_forces_dof + 3

  def _random_target(self, seed, B):
    u = _uniform((3, B), seed ^ 0x6A, 0, 0., 1., self.dev)
    dist = self.target_radius + self.target_distance * u[0]
    ang = bm.PI * 2. * u[1]
    return torch.stack([dist * torch.cos(ang), dist * torch.sin(ang),
                        self.target_height * u[2]], -1)

  def _pre_step(self, state, action):
    """`grasp.py:64-81`: scale the action, move the palm toward the last 3
    action values (at most 2 units, 15 % per step), then step the physics."""
    a = self._min_act + self._range_act * ((action + 1) / 2.)
    target_pos = a[:, -3:]
    palm = state.qp.pos[:, self.palm_idx]
    norm = torch.linalg.norm(target_pos - palm, dim=-1, keepdim=True)
    scale = torch.where(norm > 2.0, 2. / norm, torch.ones_like(norm))
    pos = state.qp.pos.clone()
    pos[:, self.palm_idx] = palm + scale * (target_pos - palm) * .15
    return QP(pos=pos, rot=state.qp.rot, vel=state.qp.vel, ang=state.qp.ang), a

  def _get_obs(self, qp, info):
    B = qp.pos.shape[0]
    inv = bm.quat_inv(qp.rot[:, self.palm_idx])[:, None]
    pos_local = bm.rotate(qp.pos - qp.pos[:, self.palm_idx:self.palm_idx + 1], inv)
    vel_local = bm.rotate(qp.vel, inv)
    ol = pos_local[:, self.object_idx]
    ol_mag = torch.linalg.norm(ol, dim=-1, keepdim=True)
    h2o = qp.pos[:, self.object_idx] - qp.pos[:, self.palm_idx]
    h2o_mag = torch.linalg.norm(h2o, dim=-1, keepdim=True)
    h2o_dir = h2o / (1e-6 + h2o_mag)
    hand_vel = qp.vel[:, self.hand_idx]
    heading = (h2o_dir * hand_vel).sum(-1, keepdim=True)
    tl = pos_local[:, self.target_idx]
    tl_mag = torch.linalg.norm(tl, dim=-1, keepdim=True)
    o2t = qp.pos[:, self.target_idx] - qp.pos[:, self.object_idx]
    o2t_mag = torch.linalg.norm(o2t, dim=-1, keepdim=True)
    o2t_dir = o2t / (1e-6 + o2t_mag)
    obj_heading = (o2t_dir * qp.vel[:, self.object_idx]).sum(-1, keepdim=True)
    contacts = _contacts(info, self.sys.num_bodies).expand(B, -1)
    return torch.cat([ol_mag, ol / (1e-6 + ol_mag), tl_mag, tl / (1e-6 + tl_mag),
                      pos_local.reshape(B, -1), vel_local.reshape(B, -1), h2o, hand_vel,
                      heading, o2t_mag, o2t_dir, obj_heading, contacts], -1)

  def _step(self, state, action, qp, info):
    dt = float(self.sys.config.dt)
    obs = self._get_obs(qp, info)
    object_pos, hand_pos = qp.pos[:, self.object_idx], qp.pos[:, self.palm_idx]
    hand_vel = qp.vel[:, self.hand_idx]
    object_rel = object_pos - hand_pos
    object_dist = torch.linalg.norm(object_rel, dim=-1, keepdim=True)
    planar = torch.linalg.norm(object_rel[:, :2], dim=-1)
    object_dir = object_rel / (1e-6 + object_dist)
    moving_to_object = .1 * dt * (hand_vel * object_dir).sum(-1)
    close_to_object = .1 * dt * 1. / (1. + planar)
    target_rel = qp.pos[:, self.target_idx] - object_pos
    target_dist = torch.linalg.norm(target_rel, dim=-1)
    target_dir = target_rel / (1e-6 + target_dist[:, None])
    moving_to_target = 1.5 * dt * (qp.vel[:, self.object_idx] * target_dir).sum(-1)
    c = _contacts(info, self.sys.num_bodies)
    touching = 0.2 * dt * (c[:, 3] + c[:, 9] + c[:, 12] + c[:, 15])
    hit = torch.where(target_dist < self.target_radius, 1.0, 0.0)
    reward = moving_to_object + close_to_object + touching + 5. * hit + moving_to_target
    metrics = _replace_metrics(state, hits=hit, touchingObject=touching,
                               movingToObject=moving_to_object,
                               movingObjectToTarget=moving_to_target,
                               closeToObject=close_to_object)
    qp, info_s = self._teleport(state, qp, hit)
    return state.replace(qp=qp, obs=obs, reward=reward, metrics=metrics, info=info_s)


class Fast(Env):
  """`brax/envs/fast.py`: the trivial unit-test env (no bodies; torch only)."""

  def __init__(self, batch_size=None, device=None, **kwargs):
    super().__init__(config=None)
    self.batch_size = batch_size
    self.dev = torch.device(device) if device is not None else torch.device('cuda')
    self.dt = 0.02

  @property
  def observation_size(self):
    return 2

  @property
  def action_size(self):
    return 1

  def reset(self, rng) -> State:
    B = self.batch_size or 1
    z = torch.zeros((B, 1), device=self.dev)
    qp = QP(pos=z, vel=z.clone(), rot=z.clone(), ang=z.clone())
    zb = torch.zeros((B,), device=self.dev)
    return State(qp=qp, obs=torch.zeros((B, 2), device=self.dev), reward=zb,
                 done=zb.clone(), metrics={}, info={})

  def step(self, state, action) -> State:
    a = torch.as_tensor(action, dtype=torch.float32, device=self.dev).reshape(-1, 1)
    vel = state.qp.vel + (a > 0).float() * self.dt
    pos = state.qp.pos + vel * self.dt
    qp = QP(pos=pos, vel=vel, rot=state.qp.rot, ang=state.qp.ang)
    obs = torch.cat([pos, vel], -1)
    return state.replace(qp=qp, obs=obs, reward=pos[:, 0])
