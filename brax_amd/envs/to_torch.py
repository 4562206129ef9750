"""`brax/envs/to_torch.py:28-64`: JaxToTorchWrapper, a gym wrapper around a
GymWrapper / VectorGymWrapper whose outputs are torch tensors.

The reference hops every leaf across DLPack (`brax/io/torch.py`): actions
torch -> JAX on the way in, observations, rewards, dones and the info tree
JAX -> torch on the way out. brax_amd's env outputs already are torch tensors
on the env's device, so the wrapper moves a leaf only when another `device` is
asked for, and its `action()` turns what a torch or numpy caller hands in
(torch tensors on any device, numpy arrays, lists) into the float32 device
tensor the fused step kernel reads. The method names, their order in `step`
and the (obs, reward, done, info) return are the reference's.
"""
from typing import Optional

import numpy as np
import torch

from brax_amd.base import QP


class JaxToTorchWrapper:
  """Wraps a `GymWrapper` or `VectorGymWrapper` (`to_torch.py:28-35`)."""

  def __init__(self, env, device: Optional[torch.device] = None):
    self.env = env
    self.device = device

  def __getattr__(self, name):
    # gym.Wrapper forwards unknown attributes (spaces, num_envs, seed, ...)
    return getattr(self.env, name)

  def _env_device(self):
    inner = self.env._env  # pylint: disable=protected-access
    return inner.unwrapped.sys.device

  def _to(self, x):
    """One leaf (or pytree of leaves) onto `device`, as `jax_to_torch` does."""
    if isinstance(x, dict):
      return {k: self._to(v) for k, v in x.items()}
    if isinstance(x, QP):
      return QP(*(self._to(v) for v in (x.pos, x.rot, x.vel, x.ang)))
    if isinstance(x, (list, tuple)):
      return type(x)(self._to(v) for v in x)
    if isinstance(x, torch.Tensor) and self.device is not None and x.device != torch.device(self.device):
      return x.to(self.device)
    return x

  def observation(self, observation):
    return self._to(observation)

  def action(self, action):
    """`torch_to_jax(action)`: here, the env device's float32 tensor."""
    dev = self._env_device()
    if isinstance(action, torch.Tensor):
      return action.to(device=dev, dtype=torch.float32)
    return torch.as_tensor(np.asarray(action, np.float32), device=dev)

  def reward(self, reward):
    return self._to(reward)

  def done(self, done):
    return self._to(done)

  def info(self, info):
    return self._to(info)

  def reset(self):
    obs = self.env.reset()
    return self.observation(obs)

  def step(self, action):
    action = self.action(action)
    obs, reward, done, info = self.env.step(action)
    obs = self.observation(obs)
    reward = self.reward(reward)
    done = self.done(done)
    info = self.info(info)
    return obs, reward, done, info
