"""`brax.envs.Env` / `State` / `Wrapper` (`brax/envs/env.py:28-102`) on MI355X.

A `PhysicsEnv` (Ant, Humanoid, HalfCheetah) steps through ONE fused kernel
launch (`bx_env_step`): System.step + observation + reward/done/metrics, plus
the EpisodeWrapper counters and the AutoResetWrapper select when those
wrappers sit directly above it (`wrappers.py` folds them into the launch).
States are batched: every leaf has a leading env axis (B, ...).
"""
import abc
import collections.abc
import ctypes as C
import dataclasses
from typing import Any, Dict

import numpy as np
import torch

from brax_amd import _native
from brax_amd import abi
from brax_amd.base import PackedQP, QP, packed_view
from brax_amd.system import System, _stream, qp_struct


@dataclasses.dataclass(frozen=True)
class State:
  """Environment state (`env.py:28-36`)."""
  qp: QP
  obs: Any
  reward: Any
  done: Any
  metrics: Dict[str, Any] = dataclasses.field(default_factory=dict)
  info: Dict[str, Any] = dataclasses.field(default_factory=dict)

  def replace(self, **kw):
    return dataclasses.replace(self, **kw)


class _Metrics(collections.abc.MutableMapping):
  """State.metrics of a kernel env step: the env's metric keys over the
  columns of the step's (B, M) metrics buffer, plus the entries carried from
  the input state. The column views are built on first access (ten views
  are ~10 µs of host time per step); a dict otherwise."""

  __slots__ = ('_m', '_keys', '_extra', '_d')

  def __init__(self, m, keys, extra):
    self._m, self._keys, self._extra, self._d = m, keys, extra, None

  def _dict(self):
    if self._d is None:
      d = dict(self._extra)
      if self._keys:
        d.update(zip(self._keys, self._m.unbind(1)))
      self._d = d
    return self._d

  def carried(self, keys):
    """The entries a next step carries over (those it does not rewrite)."""
    if self._d is None:
      return self._extra if keys == self._keys else {
          k: v for k, v in self._dict().items() if k not in keys}
    return {k: v for k, v in self._d.items() if k not in keys}

  def __getitem__(self, k):
    return self._dict()[k]

  def __setitem__(self, k, v):
    self._dict()[k] = v

  def __delitem__(self, k):
    del self._dict()[k]

  def __iter__(self):
    return iter(self._dict())

  def __len__(self):
    return len(self._dict())

  def __repr__(self):
    return repr(self._dict())


def key_to_seed(rng):
  """A jax-style PRNG key (2,) uint32, or an int, -> 64-bit seed."""
  if isinstance(rng, (int, np.integer)):
    return int(rng) & 0xFFFFFFFFFFFFFFFF
  a = np.asarray(rng.cpu() if isinstance(rng, torch.Tensor) else rng).astype(np.uint64).reshape(-1)
  if a.size >= 2:
    return (int(a[0]) << 32) | int(a[1])
  return int(a[0])


class Env(abc.ABC):
  """API for driving a brax system (`env.py:39-71`)."""

  def __init__(self, config, device=None):
    if config is not None:
      self.sys = System(config, device=device)

  @abc.abstractmethod
  def reset(self, rng) -> State:
    """Resets the environment to an initial state."""

  @abc.abstractmethod
  def step(self, state: State, action) -> State:
    """Run one timestep of the environment's dynamics."""

  @property
  def observation_size(self) -> int:
    return self.unwrapped.obs_size

  @property
  def action_size(self) -> int:
    return self.sys.num_joint_dof + self.sys.num_forces_dof

  @property
  def unwrapped(self) -> 'Env':
    return self

  # fused-chain protocol: wrappers pass their options down to the env
  def _chain_step(self, state, action, opts):
    if opts:
      raise NotImplementedError
    return self.step(state, action)


class Wrapper(Env):
  """Wraps the environment to allow modular transformations (`env.py:74-102`)."""

  def __init__(self, env: Env):
    super().__init__(config=None)
    self.env = env

  def reset(self, rng) -> State:
    return self.env.reset(rng)

  def step(self, state: State, action) -> State:
    return self.env.step(state, action)

  @property
  def observation_size(self) -> int:
    return self.env.observation_size

  @property
  def action_size(self) -> int:
    return self.env.action_size

  @property
  def unwrapped(self) -> Env:
    return self.env.unwrapped

  def __getattr__(self, name):
    if name == '__setstate__':
      raise AttributeError(name)
    return getattr(self.env, name)


class PhysicsEnv(Env):
  """An env whose step/obs/reward are one of the fused kernel's env kinds."""

  kind = 0
  metric_keys = ()
  obs_flags = 0  # abi.OBS_XY: exclude_current_positions_from_observation=False

  def __init__(self, config, batch_size=None, device=None, **kwargs):
    super().__init__(config, device=device)
    self.batch_size = batch_size
    self.coef = np.zeros(8, np.float32)
    # global id of this batch's first env: reset noise is keyed by global env
    # id, so a shard (env_offset = rank * B) resets to exactly those envs of
    # one big batch (brax_amd.distributed.shard_env)
    self.env_offset = 0

  # -------------------------------------------------------------- helpers
  def _set_sizes(self):
    """obs_size from the C ABI's own count for this kind and system
    (`bx_env_sizes`), checked against the Python metric keys."""
    p = self._params()
    o, m = C.c_int32(), C.c_int32()
    _native.check(_native.lib().bx_env_sizes(self.sys._h, C.byref(p), C.byref(o), C.byref(m)))
    if m.value != len(self.metric_keys):
      raise RuntimeError(f'{type(self).__name__}: {m.value} metrics, {len(self.metric_keys)} keys')
    self.obs_size = o.value

  def _params(self, opts=None, first_qp=None, first_obs=None):
    opts = opts or {}
    p = abi.BxEnvParams()
    p.kind = self.kind
    p.obs_size = getattr(self, 'obs_size', 0)
    p.n_metrics = len(self.metric_keys)
    p.episode_length = int(opts.get('episode_length', 0) or 0)
    p.action_repeat = int(opts.get('action_repeat', 1))
    p.auto_reset = 1 if opts.get('auto_reset') else 0
    p.obs_flags = self.obs_flags
    for i in range(8):
      p.coef[i] = float(self.coef[i])
    if first_qp is not None:
      p.first_qp = qp_struct(first_qp, True)
      p.first_obs = first_obs.data_ptr()
    return p

  def _cached_params(self, opts, first_qp, first_obs):
    """bx_env_params for this wrapper chain; rebuilt only when the options or
    the auto-reset first state change (i.e. after a reset), not per step."""
    key = (opts.get('episode_length'), opts.get('action_repeat'), bool(opts.get('auto_reset')),
           id(first_qp), None if first_obs is None else first_obs.data_ptr())
    cache = self.__dict__.setdefault('_pcache', {})
    hit = cache.get(key)
    if hit is not None and hit[1] is first_qp and hit[2] is first_obs:
      return hit[0]
    if len(cache) > 16:
      cache.clear()
    p = self._params(opts, first_qp, first_obs)
    cache[key] = (p, first_qp, first_obs)  # keeps the first state alive with its pointers
    return p

  def _alloc(self, B):
    """Every output of one env step in ONE device allocation:
    qp (B,N,16) | obs (B,O) | reward, done, steps, truncation (4,B) | metrics (B,M)."""
    N, O, M = self.sys.num_bodies, self.obs_size, max(len(self.metric_keys), 1)
    sizes = (B * N * 16, B * O, 4 * B, B * M)
    buf = torch.empty((sum(sizes),), dtype=torch.float32, device=self.sys.device)
    q, o, sc, m = buf.split(sizes)
    return packed_view(q.view(B, N, 16)), o.view(B, O), sc.view(4, B), m.view(B, M)

  def _metrics(self, met):
    return {k: met[:, i] for i, k in enumerate(self.metric_keys)}

  # -------------------------------------------------------------- reset
  def _noise_scale(self):
    # the default kinds' U[-s, s) reset noise; the body-placing kinds' reset
    # ranges are fixed by their reference envs (bx_env_reset)
    return getattr(self, 'reset_noise_scale', 0.0)

  def reset_batch(self, rng, batch_size, env_offset=None):
    """Batched `Env.reset` (e.g. `ant.py:198-220`, `reacher.py:156-174`,
    `pusher.py:178-209`, `ur5e.py:41-58`) in one C call, `bx_env_reset`:
    the env's reset draws, default_qp, the bodies its reset places, the
    target envs' streams, the reset-time Info and the observation, on the
    device.

    `rng` is one key (2,) / int: env e draws from the counter RNG keyed by
    (rng, global env id env_offset + e). A (B, 2) key batch gives every env
    its own key (`VmapWrapper.reset`). Parity with JAX threefry is unpinned
    (SURVEY §8(c)); the reset itself is pinned through `reset_from` with the
    same draws (`reset_noise`)."""
    B = int(batch_size)
    off = self.env_offset if env_offset is None else int(env_offset)
    dev = self.sys.device
    seeds = None
    if isinstance(rng, (int, np.integer)) or np.asarray(
        rng.cpu() if isinstance(rng, torch.Tensor) else rng).ndim < 2:
      seed = key_to_seed(rng)
    else:
      k = np.asarray(rng.cpu() if isinstance(rng, torch.Tensor) else rng).astype(np.uint64)
      if k.shape[0] != B:
        raise ValueError(f'{k.shape[0]} keys for {B} envs')
      seeds = torch.as_tensor(((k[:, 0] << np.uint64(32)) | k[:, -1]).view(np.int64),
                              device=dev)
      seed = 0
    qp, obs, scal, met = self._alloc(B)
    out = abi.BxEnvState()
    out.qp = qp_struct(qp, True)
    out.obs = obs.data_ptr()
    base = scal.data_ptr()
    out.reward = base
    out.done = base + 4 * B
    out.steps = base + 8 * B
    out.truncation = base + 12 * B
    out.metrics = met.data_ptr() if self.metric_keys else None
    rng = None
    if getattr(self, 'needs_rng', False):  # the target envs' per-env streams
      rng = torch.empty((B,), dtype=torch.int32, device=dev)
      out.rng = rng.data_ptr()
    p = self._params()
    _native.check(_native.lib().bx_env_reset(
        self.sys._h, C.byref(p), B, seed, off,
        None if seeds is None else C.c_void_p(seeds.data_ptr()), float(self._noise_scale()),
        C.byref(out), _stream(dev.index)))
    reward, done, _, _ = scal.unbind(0)
    return State(qp=qp, obs=obs, reward=reward, done=done, metrics=self._metrics(met),
                 info={} if rng is None else {'rng': rng})

  def reset_noise(self, rng, batch_size, env_offset=None):
    """The (qpos, qvel) that `reset_batch(rng, batch_size)` adds up, drawn
    with `bx_uniform` from the same counter stream: (B, D) each."""
    B = int(batch_size)
    off = self.env_offset if env_offset is None else int(env_offset)
    s = float(self._noise_scale())
    D = self.sys.num_joint_dof
    dev = self.sys.device
    noise = torch.empty((B, 2, D), dtype=torch.float32, device=dev)
    if noise.numel():
      _native.check(_native.lib().bx_uniform(C.c_void_p(noise.data_ptr()), noise.numel(),
                                             key_to_seed(rng), off * 2 * D, -s, s,
                                             _stream(dev.index)))
    return self.sys.default_angle().reshape(1, -1) + noise[:, 0], noise[:, 1]

  def reset_from(self, joint_angle, joint_velocity):
    """Reset state from explicit joint angles/velocities (B, num_joint_dof)."""
    qp = self.sys.default_qp(joint_angle=joint_angle, joint_velocity=joint_velocity)
    B = qp.pos.shape[0]
    obs = self.observe(qp, torch.zeros((B, self.action_size), dtype=torch.float32,
                                       device=self.sys.device))
    dev = self.sys.device
    zeros = torch.zeros((B,), dtype=torch.float32, device=dev)
    metrics = {k: torch.zeros((B,), dtype=torch.float32, device=dev) for k in self.metric_keys}
    return State(qp=qp, obs=obs, reward=zeros, done=torch.zeros_like(zeros), metrics=metrics,
                 info={})

  def observe(self, qp, action):
    """`_get_obs(qp, sys.info(qp), action)` as used by reset."""
    B = qp.pos.shape[0]
    obs = torch.empty((B, self.obs_size), dtype=torch.float32, device=self.sys.device)
    p = self._params()
    qs = qp_struct(qp, True)
    act = torch.as_tensor(action, dtype=torch.float32, device=self.sys.device).contiguous()
    _native.check(_native.lib().bx_env_observe(
        self.sys._h, C.byref(p), B, C.byref(qs), C.c_void_p(act.data_ptr()),
        act.shape[-1], act.shape[-1], C.c_void_p(obs.data_ptr()), _stream(self.sys.device.index)))
    return obs

  def reset(self, rng) -> State:
    return self.reset_batch(rng, self.batch_size or 1)

  # -------------------------------------------------------------- step
  def step(self, state: State, action) -> State:
    return self._chain_step(state, action, {})

  def _step_packed(self, state, action, opts):
    return _step_packed_impl(self, state, action, opts)

  def _chain_step(self, state, action, opts):
    dev = self.sys.device
    qin = state.qp
    if type(qin) is PackedQP:
      return self._step_packed(state, action, opts)
    B = qin.pos.shape[0]
    act = action
    if type(act) is not torch.Tensor or act.dtype != torch.float32 or not act.is_cuda:
      act = torch.as_tensor(act, dtype=torch.float32, device=dev)
    if act.dim() == 1:
      act = act.reshape(1, -1).expand(B, -1)
    if act.shape[0] != B or act.shape[1] != self.action_size or act.dim() != 2:
      raise ValueError(f'action shape {tuple(act.shape)} != {(B, self.action_size)}')
    if act.stride(-1) != 1:
      act = act.contiguous()
    auto = bool(opts.get('auto_reset'))
    first_qp = state.info.get('first_qp') if auto else None
    first_obs = state.info.get('first_obs') if auto else None
    if auto and (first_qp is None or first_obs is None):
      raise ValueError('AutoResetWrapper state lacks first_qp / first_obs')
    p = self._cached_params(opts, first_qp, first_obs)
    qp, obs, scal, met = self._alloc(B)
    sin = abi.BxEnvState()
    sin.qp = qp_struct(state.qp, True)
    done_in = _f32(state.done, dev)
    sin.done = done_in.data_ptr()
    steps_in = state.info.get('steps')
    if steps_in is not None:
      steps_in = _f32(steps_in, dev)
      sin.steps = steps_in.data_ptr()
    sout = abi.BxEnvState()
    sout.qp = qp_struct(qp, True)
    sout.obs = obs.data_ptr()
    base = scal.data_ptr()
    sout.reward = base
    sout.done = base + 4 * B
    sout.steps = base + 8 * B
    sout.truncation = base + 12 * B
    sout.metrics = met.data_ptr()
    rng_in = state.info.get('rng')
    if rng_in is None and getattr(self, 'needs_rng', False):
      rng_in = torch.zeros((B,), dtype=torch.int32, device=dev)  # a state built by hand
    rng_out = None
    if rng_in is not None:  # the target envs' per-env streams (int32 (B,))
      sin.rng = rng_in.data_ptr()
      rng_out = torch.empty_like(rng_in)
      sout.rng = rng_out.data_ptr()
    _native.check(_native.lib().bx_env_step(
        self.sys._h, C.byref(p), B, C.byref(sin), C.c_void_p(act.data_ptr()), act.stride(0),
        act.shape[1], C.byref(sout), _stream(dev.index)))
    reward, done, steps, trunc = scal.unbind(0)
    info = dict(state.info)
    if p.episode_length > 0:
      info['steps'] = steps
      info['truncation'] = trunc
    if rng_out is not None:
      info['rng'] = rng_out
    metrics = dict(state.metrics)
    if self.metric_keys:
      metrics.update(zip(self.metric_keys, met.unbind(1)))
    return State(qp=qp, obs=obs, reward=reward, done=done, metrics=metrics, info=info)


def _step_packed_impl(self, state, action, opts):
  """`_chain_step` for a packed input QP through `bx_env_step_packed`: one
  output allocation, every pointer plain, and only the views the State
  needs (the QP fields and metric columns are built on first access)."""
  dev = self.sys.device
  qbuf = state.qp._buf  # pylint: disable=protected-access
  B = qbuf.shape[0]
  act = action
  if type(act) is not torch.Tensor or act.dtype != torch.float32 or not act.is_cuda:
    act = torch.as_tensor(act, dtype=torch.float32, device=dev)
  if act.dim() == 1:
    act = act.reshape(1, -1).expand(B, -1)
  if act.dim() != 2 or act.shape[0] != B or act.shape[1] != self.action_size:
    raise ValueError(f'action shape {tuple(act.shape)} != {(B, self.action_size)}')
  if act.stride(-1) != 1:
    act = act.contiguous()
  if qbuf.dtype != torch.float32 or not qbuf.is_cuda or not qbuf.is_contiguous():
    qbuf = qbuf.contiguous().float()
  info_in = state.info
  auto = bool(opts.get('auto_reset'))
  first_qp = info_in.get('first_qp') if auto else None
  first_obs = info_in.get('first_obs') if auto else None
  if auto and (first_qp is None or first_obs is None):
    raise ValueError('AutoResetWrapper state lacks first_qp / first_obs')
  p = self._cached_params(opts, first_qp, first_obs)
  done_in = _f32(state.done, dev)
  steps_in = info_in.get('steps')
  if steps_in is not None:
    steps_in = _f32(steps_in, dev)
  rng_in = info_in.get('rng')
  if rng_in is None and getattr(self, 'needs_rng', False):
    rng_in = torch.zeros((B,), dtype=torch.int32, device=dev)  # a state built by hand
  rng_out = torch.empty_like(rng_in) if rng_in is not None else None
  N, O, M = self.sys.num_bodies, self.obs_size, len(self.metric_keys)
  out = torch.empty((B * (N * 16 + O + 4 + M),), dtype=torch.float32, device=dev)
  _native.check(_native.lib().bx_env_step_packed(
      self.sys._h, C.byref(p), B, qbuf.data_ptr(), done_in.data_ptr(),  # pylint: disable=protected-access
      None if steps_in is None else steps_in.data_ptr(),
      None if rng_in is None else rng_in.data_ptr(), act.data_ptr(), act.stride(0),
      act.shape[1], out.data_ptr(), None if rng_out is None else rng_out.data_ptr(),
      _stream(dev.index)))
  q, obs, reward, done, steps, trunc, met = torch.split(out, (B * N * 16, B * O, B, B, B, B, B * M))
  info = dict(info_in)
  if p.episode_length > 0:
    info['steps'] = steps
    info['truncation'] = trunc
  if rng_out is not None:
    info['rng'] = rng_out
  keys = self.metric_keys
  m_in = state.metrics
  extra = m_in.carried(keys) if type(m_in) is _Metrics else {
      k: v for k, v in m_in.items() if k not in keys}
  metrics = _Metrics(met.view(B, M) if M else None, keys, extra)
  return State(qp=PackedQP(q.view(B, N, 16)), obs=obs.view(B, O), reward=reward, done=done,
               metrics=metrics, info=info)


def _f32(x, dev):
  """A contiguous float32 device tensor (no copy when it already is one)."""
  if type(x) is torch.Tensor and x.dtype == torch.float32 and x.is_cuda and x.is_contiguous():
    return x
  return torch.as_tensor(x, dtype=torch.float32, device=dev).contiguous()
