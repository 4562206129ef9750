"""hipGraph-captured rollouts (`brax_amd.envs.graph.StepGraph`) on the GPU.

A graph replay runs the eager loop's kernels: every replayed step must give
the same bits as the plain Python loop of `bx_uniform` draws (at the
(step, global env id) offsets bench.py uses) and `env.step` calls, across
replays (fresh action slabs each time, from the device epoch counter) and
for an env with per-env device streams (Fetch's target teleports).
"""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _eager(env, state, steps, seed, dev, B, A, k0=0):
  from brax_amd import _native
  from brax_amd import distributed as bd
  act = torch.empty((B, A), dtype=torch.float32, device=dev)
  for k in range(steps):
    _native.check(_native.lib().bx_uniform(
        C.c_void_p(act.data_ptr()), B * A, seed, bd.action_offset(0, B, A, k0 + k, 1),
        -1.0, 1.0, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    state = env.step(state, act)
  return state


def _same(a, b):
  for name in ('obs', 'reward', 'done'):
    x, y = getattr(a, name), getattr(b, name)
    assert torch.equal(x, y), name
  for f in ('pos', 'rot', 'vel', 'ang'):
    assert torch.equal(getattr(a.qp, f), getattr(b.qp, f)), f
  assert torch.equal(a.info['steps'], b.info['steps'])
  for k in a.metrics:
    assert torch.equal(a.metrics[k], b.metrics[k]), k


def _eager_ranked(env, state, steps, seed, dev, B, A, k0, rank, world):
  from brax_amd import _native
  from brax_amd import distributed as bd
  act = torch.empty((B, A), dtype=torch.float32, device=dev)
  for k in range(steps):
    _native.check(_native.lib().bx_uniform(
        C.c_void_p(act.data_ptr()), B * A, seed, bd.action_offset(rank, B, A, k0 + k, world),
        -1.0, 1.0, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    state = env.step(state, act)
  return state


@pytest.mark.parametrize('name,B,K,draw', [('ant', 512, 5, 'batched'), ('ant', 512, 5, 'per_step'),
                                           ('humanoid', 256, 3, 'batched'),
                                           ('fetch', 128, 4, 'batched'),
                                           ('ant', 64, 1, 'batched')])
def test_graph_replays_match_eager_loop(dev, name, B, K, draw):
  from brax_amd import envs
  from brax_amd import distributed as bd
  from brax_amd.envs.graph import StepGraph
  env = envs.create(name, batch_size=B, episode_length=7, auto_reset=True, device=dev)
  A = env.action_size
  st0 = env.reset(np.array([0, 11], np.uint32))
  # 2 replays of K steps: covers an auto-reset (episode length 7) and the
  # epoch counter's second slab set
  ref = _eager(env, st0, 2 * K, 5, dev, B, A, k0=3)
  g = StepGraph(env, st0, K, seed=5, offset=bd.action_offset(0, B, A, 3, 1), step_stride=B * A,
                draw=draw)
  out = g.replay()
  mid = _eager(env, st0, K, 5, dev, B, A, k0=3)
  _same(out, mid)
  out = g.replay()
  torch.cuda.synchronize()
  _same(out, ref)
  assert g.epoch == 2
  if 'rng' in st0.info:
    assert torch.equal(out.info['rng'], ref.info['rng'])


@pytest.mark.parametrize('draw', ['batched', 'per_step'])
def test_graph_rank_slabs_match_eager_loop(dev, draw):
  """Rank 1 of a world of 2: the job's per-step stride (world x B x A) and
  the rank's row offset; the one-launch slab draw gives every step the bits
  of the eager loop's bx_uniform at action_offset(1, B, A, step, 2)."""
  from brax_amd import envs
  from brax_amd import distributed as bd
  from brax_amd.envs.graph import StepGraph
  B, K, world, rank, k0 = 128, 4, 2, 1, 6
  env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  A = env.action_size
  bd.shard_env(env, rank, B)
  st0 = env.reset(np.array([0, 4], np.uint32))
  ref = _eager_ranked(env, st0, 3 * K, 2, dev, B, A, k0, rank, world)
  g = StepGraph(env, st0, K, seed=2, offset=bd.action_offset(rank, B, A, k0, world),
                step_stride=world * B * A, draw=draw)
  for _ in range(3):
    out = g.replay()
  torch.cuda.synchronize()
  _same(out, ref)


def test_graph_target_env_without_rng_advances_stream(dev):
  """A hand-built Fetch state without info['rng']: the graph makes the
  stream a static input, so replays continue it like the eager loop (which
  starts a zero stream once and carries it)."""
  from brax_amd import envs
  from brax_amd.envs.graph import StepGraph
  B, K = 64, 3
  env = envs.create('fetch', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  st0 = env.reset(np.array([0, 2], np.uint32))
  info = {k: v for k, v in st0.info.items() if k != 'rng'}
  st0 = st0.replace(info=info)
  g = StepGraph(env, st0, K, seed=7)
  g.replay()
  out = g.replay()
  st = st0.replace(info=dict(info, rng=torch.zeros((B,), dtype=torch.int32, device=dev)))
  ref = _eager(env, st, 2 * K, 7, dev, B, env.action_size)
  torch.cuda.synchronize()
  _same(out, ref)
  assert torch.equal(out.info['rng'], ref.info['rng'])


def test_graph_hook_and_exchange_accumulate(dev):
  """The per-step hook is recorded into the graph: an EpisodeExchange-style
  device sum over a replayed rollout equals the eager loop's."""
  from brax_amd import envs
  from brax_amd.envs.graph import StepGraph
  B, K = 256, 4
  env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  st0 = env.reset(np.array([0, 3], np.uint32))
  acc_g = torch.zeros((2, B), device=dev)

  def hook(st):
    acc_g[0].add_(st.reward)
    acc_g[1].add_(st.done)
  g = StepGraph(env, st0, K, seed=9, hook=hook)
  g.replay()
  g.replay()
  acc_e = torch.zeros((2, B), device=dev)
  from brax_amd import _native
  act = torch.empty((B, env.action_size), device=dev)
  st = st0
  for k in range(2 * K):
    _native.check(_native.lib().bx_uniform(
        C.c_void_p(act.data_ptr()), act.numel(), 9, k * act.numel(), -1.0, 1.0,
        C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    st = env.step(st, act)
    acc_e[0].add_(st.reward)
    acc_e[1].add_(st.done)
  torch.cuda.synchronize()
  assert torch.equal(acc_g, acc_e)
