"""Env wrappers (`brax/envs/wrappers.py:31-148`).

EpisodeWrapper and AutoResetWrapper keep the reference's semantics exactly;
when they wrap a PhysicsEnv (optionally through Vector/VmapWrapper) their
logic runs INSIDE the fused env-step kernel (one launch per step). Above any
other env they run as device tensor ops with the same semantics.
"""
import dataclasses
from typing import Dict, Optional

import numpy as np
import torch

from brax_amd.envs.env import Env, State, Wrapper, key_to_seed


def wrap_for_training(env: Env, episode_length: int = 1000, action_repeat: int = 1):
  """`wrappers.py:31-55`: Episode -> Vmap -> AutoReset."""
  env = EpisodeWrapper(env, episode_length, action_repeat)
  env = VmapWrapper(env)
  return AutoResetWrapper(env)


class VectorWrapper(Wrapper):
  """`wrappers.py:58-70`: batches `batch_size` envs (states are batched natively)."""

  def __init__(self, env: Env, batch_size: int):
    super().__init__(env)
    self.batch_size = batch_size

  def reset(self, rng) -> State:
    u = self.env.unwrapped
    if hasattr(u, 'reset_batch') and self.env is u:
      return u.reset_batch(rng, self.batch_size)
    return _reset_batch(self.env, rng, self.batch_size)

  def step(self, state, action):
    return self.env.step(state, action)

  def _chain_step(self, state, action, opts):
    return self.env._chain_step(state, action, opts)  # pylint: disable=protected-access


class VmapWrapper(Wrapper):
  """`wrappers.py:73-80`: rng carries a leading batch axis (B, 2); env e
  resets from its own key rng[e], as `jax.vmap(env.reset)(rng)` does."""

  def reset(self, rng) -> State:
    rng = np.asarray(rng.cpu() if isinstance(rng, torch.Tensor) else rng)
    if rng.ndim != 2:
      return _reset_batch(self.env, rng, 1)
    return _reset_batch(self.env, rng, rng.shape[0])

  def step(self, state, action):
    return self.env.step(state, action)

  def _chain_step(self, state, action, opts):
    return self.env._chain_step(state, action, opts)  # pylint: disable=protected-access


def _reset_batch(env, rng, batch_size):
  if isinstance(env, EpisodeWrapper):
    st = _reset_batch(env.env, rng, batch_size)
    return env._add_counters(st)  # pylint: disable=protected-access
  u = env.unwrapped
  if env is u and hasattr(u, 'reset_batch'):
    return u.reset_batch(rng, batch_size)
  if isinstance(env, Wrapper):
    return _reset_batch(env.env, rng, batch_size)
  return env.reset(rng)


class _ScaledConfigSystem:
  """EpisodeWrapper.sys (`wrappers.py:92-95`): the reference deep-copies the
  env's System and multiplies its *config's* dt and substeps by
  action_repeat ("for proper video speed"); the copy's integrator keeps the
  original step. Here: the env's System, with a scaled copy of its config."""

  def __init__(self, sys_, action_repeat):
    import copy  # pylint: disable=import-outside-toplevel
    self._sys = sys_
    self.config = copy.deepcopy(sys_.config)
    self.config.dt *= action_repeat
    self.config.substeps *= action_repeat

  def __getattr__(self, name):
    return getattr(self._sys, name)


class EpisodeWrapper(Wrapper):
  """`wrappers.py:83-120`: step counter, truncation and episode-length done."""

  def __init__(self, env: Env, episode_length: int, action_repeat: int):
    super().__init__(env)
    self.episode_length = episode_length
    self.action_repeat = action_repeat
    if hasattr(env, 'sys'):
      self.sys = _ScaledConfigSystem(env.sys, action_repeat)

  def _add_counters(self, state):
    z = torch.zeros_like(torch.as_tensor(state.done))
    info = dict(state.info)
    info['steps'] = z
    info['truncation'] = torch.zeros_like(z)
    return state.replace(info=info)

  def reset(self, rng) -> State:
    return self._add_counters(self.env.reset(rng))

  def step(self, state, action):
    return self._chain_step(state, action, {})

  def _chain_step(self, state, action, opts):
    mine = dict(opts, episode_length=self.episode_length, action_repeat=self.action_repeat)
    try:
      return self.env._chain_step(state, action, mine)  # pylint: disable=protected-access
    except NotImplementedError:
      if opts:
        raise
    # generic device-tensor path (reference semantics)
    rewards = []
    for _ in range(self.action_repeat):
      state = self.env.step(state, action)
      rewards.append(state.reward)
    state = state.replace(reward=torch.stack(rewards).sum(0))
    steps = state.info['steps'] + self.action_repeat
    one = torch.ones_like(state.done)
    zero = torch.zeros_like(state.done)
    done = torch.where(steps >= self.episode_length, one, state.done)
    info = dict(state.info)
    info['truncation'] = torch.where(steps >= self.episode_length, 1 - state.done, zero)
    info['steps'] = steps
    return state.replace(done=done, info=info)


class AutoResetWrapper(Wrapper):
  """`wrappers.py:123-148`: done envs restart from the stored first state."""

  def reset(self, rng) -> State:
    state = self.env.reset(rng)
    info = dict(state.info)
    info['first_qp'] = state.qp
    info['first_obs'] = state.obs
    return state.replace(info=info)

  def step(self, state, action):
    try:
      return self.env._chain_step(state, action, {'auto_reset': True})  # pylint: disable=protected-access
    except NotImplementedError:
      pass
    info = dict(state.info)
    if 'steps' in info:
      info['steps'] = torch.where(state.done != 0, torch.zeros_like(info['steps']), info['steps'])
    state = state.replace(done=torch.zeros_like(state.done), info=info)
    state = self.env.step(state, action)
    return self._select(state)

  @staticmethod
  def _select(state):
    done = state.done != 0
    fq, fo = state.info['first_qp'], state.info['first_obs']
    d3 = done.reshape(-1, 1, 1)
    from brax_amd.base import QP  # pylint: disable=import-outside-toplevel
    qp = QP(pos=torch.where(d3, fq.pos, state.qp.pos), rot=torch.where(d3, fq.rot, state.qp.rot),
            vel=torch.where(d3, fq.vel, state.qp.vel), ang=torch.where(d3, fq.ang, state.qp.ang))
    obs = torch.where(done.reshape(-1, 1), fo, state.obs)
    return state.replace(qp=qp, obs=obs)


@dataclasses.dataclass(frozen=True)
class EvalMetrics:
  """`wrappers.py:150-166`: per-episode aggregated metrics."""
  episode_metrics: Dict[str, torch.Tensor]
  active_episodes: torch.Tensor
  episode_steps: torch.Tensor


class EvalWrapper(Wrapper):
  """`wrappers.py:169-203`: episode metrics summed while an episode is active."""

  def reset(self, rng) -> State:
    st = self.env.reset(rng)
    metrics = dict(st.metrics)
    metrics['reward'] = st.reward
    em = EvalMetrics(episode_metrics={k: torch.zeros_like(v) for k, v in metrics.items()},
                     active_episodes=torch.ones_like(st.reward),
                     episode_steps=torch.zeros_like(st.reward))
    info = dict(st.info)
    info['eval_metrics'] = em
    return st.replace(metrics=metrics, info=info)

  def step(self, state: State, action) -> State:
    em = state.info['eval_metrics']
    if not isinstance(em, EvalMetrics):
      raise ValueError(f'Incorrect type for state_metrics: {type(em)}')
    info = dict(state.info)
    del info['eval_metrics']
    nstate = self.env.step(state.replace(info=info), action)
    metrics = dict(nstate.metrics)
    metrics['reward'] = nstate.reward
    episode_steps = torch.where(em.active_episodes != 0, nstate.info['steps'], em.episode_steps)
    episode_metrics = {k: em.episode_metrics[k] + metrics[k] * em.active_episodes
                       for k in em.episode_metrics}
    active = em.active_episodes * (1 - nstate.done)
    ninfo = dict(nstate.info)
    ninfo['eval_metrics'] = EvalMetrics(episode_metrics=episode_metrics, active_episodes=active,
                                        episode_steps=episode_steps)
    return nstate.replace(metrics=metrics, info=ninfo)


# ---------------------------------------------------------------------------
# gym-API adapters (`wrappers.py:206-337`) -- gym itself is not a dependency:
# spaces are plain Box descriptions; outputs stay device tensors (the torch
# side, the reference's JaxToTorchWrapper, is `brax_amd.envs.to_torch`).
# ---------------------------------------------------------------------------

@dataclasses.dataclass(frozen=True)
class Box:
  """A gym.spaces.Box-like description (low, high, shape, dtype)."""
  low: np.ndarray
  high: np.ndarray
  shape: tuple
  dtype: str = 'float32'


def _box(n, bound, batch=None):
  shape = (n,) if batch is None else (batch, n)
  high = np.full(shape, bound, np.float32)
  return Box(low=-high, high=high, shape=shape)


def split_key(key):
  """Two child keys of a (2,) uint32 key (the reference's
  `jp.random_split(key)`; threefry parity is unpinned)."""
  s = key_to_seed(key)
  out = []
  for i in (1, 2):
    z = (s + 0x9E3779B97F4A7C15 * i) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    z ^= z >> 31
    out.append(np.array([z >> 32, z & 0xFFFFFFFF], np.uint32))
  return out


class GymWrapper:
  """`wrappers.py:206-262`: one Brax env behind the gym Env API."""

  def __init__(self, env: Env, seed: int = 0, backend: Optional[str] = None):
    self._env = env
    self.metadata = {'render.modes': ['human', 'rgb_array'],
                     'video.frames_per_second': 1 / float(env.sys.config.dt)}
    self.seed(seed)
    self.backend = backend
    self._state = None
    self.observation_space = _box(env.observation_size, np.inf)
    self.action_space = _box(env.action_size, 1.0)

  def reset(self):
    self._key, key2 = split_key(self._key)
    self._state = self._env.reset(key2)
    return self._state.obs

  def step(self, action):
    self._state = self._env.step(self._state, action)
    info = {**self._state.metrics, **self._state.info}
    return self._state.obs, self._state.reward, self._state.done, info

  def seed(self, seed: int = 0):
    self._key = np.array([0, seed], np.uint32)  # jax.random.PRNGKey(seed) layout

  def render(self, mode='human'):
    raise NotImplementedError('rendering (brax.io) is outside the MI355X path')


class VectorGymWrapper(GymWrapper):
  """`wrappers.py:265-337`: a batched Brax env behind the gym VectorEnv API."""

  def __init__(self, env: Env, seed: int = 0, backend: Optional[str] = None):
    if not hasattr(env, 'batch_size') or not env.batch_size:
      raise ValueError('underlying env must be batched')
    super().__init__(env, seed, backend)
    self.num_envs = env.batch_size
    self.single_observation_space = self.observation_space
    self.single_action_space = self.action_space
    self.observation_space = _box(env.observation_size, np.inf, self.num_envs)
    self.action_space = _box(env.action_size, 1.0, self.num_envs)
