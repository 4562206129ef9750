"""Env wrappers (`brax/envs/wrappers.py:31-148`).

EpisodeWrapper and AutoResetWrapper keep the reference's semantics exactly;
when they wrap a PhysicsEnv (optionally through Vector/VmapWrapper) their
logic runs INSIDE the fused env-step kernel (one launch per step). Above any
other env they run as device tensor ops with the same semantics.
"""
import torch

from brax_amd.envs.env import Env, State, Wrapper


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
  """`wrappers.py:73-80`: rng carries a leading batch axis (B, 2)."""

  def reset(self, rng) -> State:
    rng = torch.as_tensor(rng)
    B = rng.shape[0] if rng.dim() == 2 else 1
    return _reset_batch(self.env, rng[0] if rng.dim() == 2 else rng, B)

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


class EpisodeWrapper(Wrapper):
  """`wrappers.py:83-120`: step counter, truncation and episode-length done."""

  def __init__(self, env: Env, episode_length: int, action_repeat: int):
    super().__init__(env)
    self.episode_length = episode_length
    self.action_repeat = action_repeat

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
