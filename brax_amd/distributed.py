"""Multi-GPU sharding of env batches.

The physics never crosses GPUs: rank r owns the contiguous global env ids
[r*B, (r+1)*B) and its reset/action RNG streams are keyed by rank. The only
collective is the per-step (reward, done) all-gather over RCCL (backend
"nccl" on ROCm) — or gloo for host tensors in tests. The reference's analogue
is `jax.pmap` env sharding (`agents/ppo/train.py:112,276-283`).
"""
import numpy as np
import torch
import torch.distributed as dist


def env_range(rank: int, envs_per_rank: int):
  """Global env ids owned by `rank`."""
  return rank * envs_per_rank, (rank + 1) * envs_per_rank


def rank_key(rng, rank: int):
  """Per-rank reset key: (seed_hi ^ rank, seed_lo) keeps streams disjoint."""
  k = np.asarray(rng, np.uint32).reshape(-1)
  hi = int(k[0]) if k.size > 1 else 0
  lo = int(k[-1])
  return np.array([(hi ^ (0x9E37 * (rank + 1))) & 0xFFFFFFFF, lo], np.uint32)


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
