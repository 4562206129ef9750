"""World-size-2 gloo rehearsal of the multi-GPU path (no GPU needed)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from brax_amd import distributed as bd


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _worker(rank, world, port, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  B = 5
  lo, hi = bd.env_range(rank, B)
  reward = torch.arange(lo, hi, dtype=torch.float32)
  done = (torch.arange(lo, hi) % 2).float()
  ex = bd.EpisodeExchange(B, 'cpu', every=3)
  # the step's (reward, done) rows of one (4, B) buffer, as an env step returns them
  scal = torch.stack([reward, done, torch.zeros(B), torch.zeros(B)])
  assert ex(*scal.unbind(0)[:2]) is None and ex(reward, done) is None
  out = ex(*scal.unbind(0)[:2])  # the third step: the episodic gather
  out = out.numpy().copy()
  left = float(ex.acc.abs().sum())
  # a graph-replayed rollout's split: device sums per step, host count after
  # each replay of 2 steps, period 4 (the bench's exchange_period logic)
  ex = bd.EpisodeExchange(B, 'cpu', every=bd.exchange_period(1000, 4, replay=2))
  assert ex.every == 4
  for _ in range(2):
    ex.accumulate(*scal.unbind(0)[:2])
  assert ex.advance(2) is None  # k = 2: mid-period
  for _ in range(2):
    ex.accumulate(reward, done)
  out2 = ex.advance(2)  # k = 4: the episodic gather
  np.testing.assert_array_equal(out2.numpy()[:, 0], 4 * out[:, 0] / 3)
  assert ex.flushes == 1
  try:
    ex.advance(3)  # a period boundary inside the replay: refused
    raise AssertionError('advance(3) with every=4 must raise')
  except ValueError:
    pass
  ex.reset()
  assert ex.k == 0 and ex.flushes == 0 and float(ex.acc.abs().sum()) == 0
  q.put((rank, out, bd.action_offset(rank, B, 8, step=3, world=world), left))
  dist.barrier()
  dist.destroy_process_group()


def test_episode_allgather_world2():
  world = 2
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = [q.get(timeout=120) for _ in range(world)]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  res.sort()
  expect_r = np.arange(10, dtype=np.float32).reshape(2, 5)
  for rank, out, key, left in res:
    # three steps summed per env, every rank's envs in global order
    assert out.shape == (2, 2, 5)
    np.testing.assert_array_equal(out[:, 0], 3 * expect_r)
    np.testing.assert_array_equal(out[:, 1], 3 * (expect_r % 2))
    assert left == 0.0  # the sums restart after the exchange
  # rank r's action rows of step 3 continue rank r-1's in the global stream
  assert res[1][2] - res[0][2] == 5 * 8


def test_exchange_period():
  assert bd.exchange_period(1000, 20, 20) == 20  # the driver's 20-step run: one gather
  assert bd.exchange_period(1000, 1000, 50) == 1000
  assert bd.exchange_period(1000, 5000, 50) == 1000
  assert bd.exchange_period(1000, 30, 20) == 20
  assert bd.exchange_period(7, 3, 5) == 5


def test_env_range():
  assert bd.env_range(0, 4096) == (0, 4096)
  assert bd.env_range(3, 4096) == (12288, 16384)


def test_action_offsets_tile_the_global_stream():
  """Per-rank action slabs keyed by (step, global env id) cover exactly the
  rows one big batch of world*B envs draws at that step."""
  B, A = 4096, 8
  for world in (1, 2, 4, 8):
    for step in (0, 1, 17):
      offs = [bd.action_offset(r, B, A, step, world) for r in range(world)]
      big = bd.action_offset(0, world * B, A, step, 1)
      assert offs == [big + r * B * A for r in range(world)]


class _Env:
  def __init__(self):
    self.env_offset = 0

  @property
  def unwrapped(self):
    return self


def test_shard_env_sets_global_offset():
  e = bd.shard_env(_Env(), 3, 4096)
  assert e.env_offset == 3 * 4096
