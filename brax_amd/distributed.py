"""Multi-GPU sharding of env batches.

The physics never crosses GPUs: rank r owns the contiguous global env ids
[r*B, (r+1)*B). Reset noise and synthetic actions are keyed by GLOBAL env id
(one shared seed, `env_offset = r*B`), so N shards of B envs hold exactly the
states of one batch of N*B envs, whatever the GPU count. The only collective
is the episodic (reward, done) all-gather over RCCL (backend "nccl" on ROCm) —
or gloo for host tensors in tests: every rank sums its envs' rewards and done
flags on the device each step and the sums are gathered once per episode
length, as the reference's trainers reduce episode metrics once per
evaluation (`agents/ppo/train.py:276-283` shards the envs by global index the
same way). A per-step gather would put an RCCL round trip (tens of µs over
xGMI) on every 36 µs step.
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


def exchange_period(episode_length: int, timed_steps: int, replay: int = 1) -> int:
  """Steps between episodic all-gathers in a timed run: the episode length,
  or the timed step count when that is shorter (so a short timed region
  still holds at least one collective), rounded down to a multiple of the
  graph replay length (`EpisodeExchange.advance` counts whole replays)."""
  replay = max(int(replay), 1)
  p = min(int(episode_length), int(timed_steps))
  return max(p - p % replay, replay)


class EpisodeExchange:
  """Episodic exchange of every rank's per-env (reward, done).

  Each call adds the step's (reward, done) into a (2, B) device sum (one
  add: the env step returns both rows of one (4, B) buffer); every `every`
  calls (the episode length) the sums of all ranks are all-gathered into
  (world, 2, B) (RCCL on device tensors, gloo on host ones), returned, and
  reset. Other calls return None."""

  def __init__(self, envs_per_rank: int, device, every: int = 1000, group=None):
    self.group = group
    self.world = dist.get_world_size(group)
    self.B = envs_per_rank
    self.every = max(int(every), 1)
    self.k = 0
    self.acc = torch.zeros((2, envs_per_rank), dtype=torch.float32, device=device)
    self.out = torch.empty((self.world, 2, envs_per_rank), dtype=torch.float32, device=device)
    self._nccl = dist.get_backend(group) == 'nccl'
    self.flushes = 0  # all-gathers done (bench.py reports those in its timed region)

  def __call__(self, reward, done):
    self.accumulate(reward, done)
    self.k += 1
    return self.flush() if self.k % self.every == 0 else None

  def accumulate(self, reward, done):
    """The device half of a call: adds the step's (reward, done) to the
    sums. Stream-ordered device work only, so a graph-captured rollout
    (`brax_amd.envs.graph.StepGraph`) records it as its per-step hook and
    calls `advance` on the host after each replay."""
    B = self.B
    if (reward.dtype == done.dtype == torch.float32 and reward.is_contiguous() and
        reward.device == self.acc.device and done.data_ptr() == reward.data_ptr() + 4 * B):
      self.acc.add_(reward.as_strided((2, B), (B, 1)))  # both rows of the step's buffer
    else:
      self.acc[0].add_(reward.float())
      self.acc[1].add_(done.float())

  def accumulate_steps(self, reward, done):
    """A rollout's K steps at once: (K, B) rewards and dones summed over the
    steps into the sums (the device half of K calls; the float sum's order
    is torch's reduction, not step by step)."""
    self.acc[0].add_(reward.sum(0))
    self.acc[1].add_(done.sum(0))

  def reset(self):
    """Zeroes the sums and the step count (e.g. at the start of a timed
    region, so its exchange periods start there)."""
    self.acc.zero_()
    self.k = 0
    self.flushes = 0

  def advance(self, n):
    """Counts `n` steps accumulated by a replayed graph; flushes (and
    returns the gathered sums) when they complete an exchange period. The
    device sums already hold all n steps, so a period boundary must fall at
    the end of the n steps: `every` must be a multiple of n and the count so
    far too, else ValueError (a flush inside the replay would gather steps
    past the boundary)."""
    n = int(n)
    if n < 1 or self.every % n or self.k % n:
      raise ValueError(f'exchange period {self.every} and step count {self.k} must be '
                       f'multiples of the replay length {n}')
    self.k += n
    return self.flush() if self.k % self.every == 0 else None

  def flush(self):
    """All-gathers the sums since the last exchange, resets them and returns
    the gathered (world, 2, B) sums (a fresh tensor per flush)."""
    if self._nccl or self.acc.device.type == 'cpu':
      # one all_gather_into_tensor into the ranks' sums concatenated along
      # dim 0: RCCL's call on the device, and the same call on gloo with host
      # tensors, which is how the CPU tests run this path
      flat = torch.empty((self.world * 2, self.B), dtype=self.acc.dtype, device=self.acc.device)
      dist.all_gather_into_tensor(flat, self.acc, group=self.group)
      out = flat.view(self.world, 2, self.B)
    else:  # gloo with device tensors (the one-GPU rehearsal of the N-rank bench)
      parts = list(torch.empty_like(self.out).unbind(0))
      dist.all_gather(parts, self.acc.clone(), group=self.group)
      out = torch.stack(parts)
    self.out = out
    self.acc.zero_()
    self.flushes += 1
    return out
