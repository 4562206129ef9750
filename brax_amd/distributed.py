"""Multi-GPU sharding of env batches.

The physics never crosses GPUs: rank r owns the contiguous global env ids
[r*B, (r+1)*B). Reset noise and synthetic actions are keyed by GLOBAL env id
(one shared seed, `env_offset = r*B`), so N shards of B envs hold exactly the
states of one batch of N*B envs, whatever the GPU count. The only collective
is the per-step (reward, done) all-gather over RCCL (backend "nccl" on ROCm) —
or gloo for host tensors in tests. The reference's analogue is `jax.pmap` env
sharding by global index (`agents/ppo/train.py:276-283`).
"""
import numpy as np
import torch
import torch.distributed as dist


def env_range(rank: int, envs_per_rank: int):
  """Global env ids owned by `rank`."""
  return rank * envs_per_rank, (rank + 1) * envs_per_rank


def shard_env(env, rank: int, envs_per_rank: int):
  """Makes `env` (any wrapper chain over a kernel env) the shard of global
  envs [rank*B, (rank+1)*B): its resets draw the noise of those env ids."""
  env.unwrapped.env_offset = env_range(rank, envs_per_rank)[0]
  return env


def action_offset(rank: int, envs_per_rank: int, action_size: int, step: int = 0,
                  world: int = 1):
  """`bx_uniform` offset of rank r's (B, A) action slab at `step` in a
  stream keyed by (step, global env id, action index): slab t of the whole
  job starts at t * world * B * A, rank r's rows at r * B * A within it."""
  return (step * world + rank) * envs_per_rank * action_size


class EpisodeExchange:
  """All-gathers every rank's per-env (reward, done) into (world, 2, B)."""

  def __init__(self, envs_per_rank: int, device, group=None):
    self.group = group
    self.world = dist.get_world_size(group)
    self.B = envs_per_rank
    self.out = torch.empty((self.world, 2, envs_per_rank), dtype=torch.float32, device=device)
    self._nccl = dist.get_backend(group) == 'nccl'

  def __call__(self, reward, done):
    rd = torch.stack([reward.float(), done.float()])
    if self._nccl:
      dist.all_gather_into_tensor(self.out, rd, group=self.group)
    else:
      parts = list(self.out.unbind(0))
      dist.all_gather(parts, rd, group=self.group)
      self.out = torch.stack(parts)
    return self.out
