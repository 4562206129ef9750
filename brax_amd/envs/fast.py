"""Fast (`brax/envs/fast.py`): the reference's trivial unit-test env. It has
no bodies, so there is no physics to run: a 1-d point whose velocity grows by
dt while the action is positive; device tensor ops only."""
import torch

from brax_amd.base import QP
from brax_amd.envs.env import Env, State


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
