"""Open-loop rollouts (`brax_amd.envs.rollout.rollout`, one
`bx_env_rollout_packed` launch for K steps) against K chained `env.step`
calls on the same actions: every step's state, observation, reward, done,
episode counters, metrics and per-env stream must be bit-identical, across
auto-resets (short episodes), action repeats and every kernel family (the
SINGLE kernels at one and two rows per lane, the item loops, the env
programs with pre-step actions and per-env streams)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _check(env, st0, acts):
  from brax_amd.envs.rollout import rollout
  final, tr = rollout(env, st0, acts)
  st = st0
  for t in range(acts.shape[0]):
    st = env.step(st, acts[t])
    q = torch.cat([st.qp.pos, st.qp.rot, st.qp.vel, st.qp.ang], -1)
    assert torch.equal(tr.qp[t][..., :13], q), t
    assert torch.equal(tr.obs[t], st.obs), t
    assert torch.equal(tr.reward[t], st.reward), t
    assert torch.equal(tr.done[t], st.done), t
    if 'steps' in st.info:
      assert torch.equal(tr.steps[t], st.info['steps']), t
      assert torch.equal(tr.truncation[t], st.info['truncation']), t
    for i, k in enumerate(tr.metric_keys):
      assert torch.equal(tr.metrics[t][:, i], st.metrics[k]), (t, k)
    if 'rng' in st.info:
      assert torch.equal(tr.rng[t], st.info['rng']), t
  assert torch.equal(final.qp.pos, st.qp.pos) and torch.equal(final.obs, st.obs)
  assert torch.equal(final.done, st.done)
  return tr


@pytest.mark.parametrize('name,B,K,ep,ar', [
    ('ant', 256, 12, 5, 1), ('ant', 64, 9, 4, 2), ('humanoid', 128, 10, 6, 1),
    ('humanoidstandup', 64, 6, 4, 1), ('halfcheetah', 64, 8, 3, 1), ('pusher', 32, 5, 3, 1),
    ('fetch', 64, 7, 3, 1), ('grasp', 32, 5, 3, 1), ('reacherangle', 64, 8, 3, 1),
    ('swimmer', 64, 8, 3, 1), ('hopper', 64, 12, 4, 1), ('ur5e', 64, 6, 3, 2)])
def test_rollout_matches_chained_steps(dev, name, B, K, ep, ar):
  from brax_amd import envs
  env = envs.create(name, batch_size=B, episode_length=ep, action_repeat=ar, auto_reset=True,
                    device=dev)
  st0 = env.reset(np.array([2, 9], np.uint32))
  g = torch.Generator(device='cpu').manual_seed(4)
  acts = (torch.rand((K, B, env.action_size), generator=g) * 2 - 1).to(dev)
  tr = _check(env, st0, acts)
  assert float(tr.done.sum()) > 0  # the episodes ended inside the rollout
  torch.cuda.synchronize()


def test_rollout_without_wrappers_and_strided_actions(dev):
  """No Episode / AutoReset wrappers (the bare env), and a (K, B, A) view
  with a padded row stride."""
  from brax_amd import envs
  env = envs.create('ant', batch_size=64, episode_length=None, auto_reset=False, device=dev)
  st0 = env.reset(np.array([1, 1], np.uint32))
  base = (torch.rand((6, 64, 10), device=dev) * 2 - 1)
  acts = base[..., :8]
  assert acts.stride(1) == 10
  _check(env, st0, acts)


def test_rollout_full_batch_ant(dev):
  """BASELINE configs[1]'s batch: 4,096 Ant envs, 20 steps in one launch."""
  from brax_amd import envs
  env = envs.create('ant', batch_size=4096, episode_length=1000, auto_reset=True, device=dev)
  st0 = env.reset(np.array([0, 0x5EED], np.uint32))
  acts = torch.rand((20, 4096, 8), device=dev) * 2 - 1
  _check(env, st0, acts)


@pytest.mark.parametrize('runner', ['graph', 'direct'])
def test_rollout_graph_matches_eager_loop(dev, runner):
  """RolloutGraph replays and RolloutRunner runs (one slab draw + one
  rollout launch per K steps) step on the eager loop's bits: bx_uniform at
  action_offset(rank, B, A, step, world) per step, env.step per step (rank 1
  of a world of 2)."""
  import ctypes as C
  from brax_amd import _native, envs
  from brax_amd import distributed as bd
  from brax_amd.envs.rollout import RolloutGraph, RolloutRunner
  B, K, world, rank, k0 = 128, 5, 2, 1, 3
  env = envs.create('ant', batch_size=B, episode_length=7, auto_reset=True, device=dev)
  A = env.action_size
  bd.shard_env(env, rank, B)
  st0 = env.reset(np.array([0, 4], np.uint32))
  acc = torch.zeros((2, B), device=dev)

  def hook(tr):
    acc[0].add_(tr.reward.sum(0))
    acc[1].add_(tr.done.sum(0))
  kw = dict(seed=3, offset=bd.action_offset(rank, B, A, k0, world), step_stride=world * B * A,
            hook=hook)
  if runner == 'graph':
    g = RolloutGraph(env, st0, K, **kw)
    for _ in range(2):
      out, tr = g.replay()
  else:
    g = RolloutRunner(env, st0, K, **kw)
    for _ in range(2):
      g.run()
    out, tr = g.state(), g.trajectory()
  act = torch.empty((B, A), dtype=torch.float32, device=dev)
  st = st0
  done_sum = torch.zeros((B,), device=dev)
  for k in range(2 * K):
    _native.check(_native.lib().bx_uniform(
        C.c_void_p(act.data_ptr()), B * A, 3, bd.action_offset(rank, B, A, k0 + k, world),
        -1.0, 1.0, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    st = env.step(st, act)
    done_sum += st.done
  torch.cuda.synchronize()
  assert torch.equal(out.qp.pos, st.qp.pos) and torch.equal(out.obs, st.obs)
  assert torch.equal(out.info['steps'], st.info['steps'])
  assert torch.equal(tr.done[K - 1], st.done)
  assert torch.equal(acc[1], done_sum)  # 0 / 1 sums are exact in any order


def test_rollout_wide_batch_ant(dev):
  """Past one wave per SIMD (16,384 envs: 4 waves per SIMD) the Ant step and
  rollout launches take the register-capped kernels: the same bits."""
  from brax_amd import envs
  env = envs.create('ant', batch_size=16384, episode_length=1000, auto_reset=True, device=dev)
  st0 = env.reset(np.array([0, 0x5EED], np.uint32))
  acts = torch.rand((4, 16384, 8), device=dev) * 2 - 1
  _check(env, st0, acts)


@pytest.mark.parametrize('name', ['ant', 'fetch'])
def test_env_speed_like_reference(dev, name):
  """The reference's own speed test (brax/tests/env_test.py:30-75): 128 envs,
  episode_length 1000 (auto-reset off for Ant's early termination), a
  `lax.scan` of 1,000 zero-action `env.step`s from reset; every env is done
  at the end and the rate beats 0.99 x 1000 steps/s. Here the scan is one
  `rollout` launch of 1,000 steps."""
  import time
  from brax_amd import envs
  from brax_amd.envs.rollout import rollout
  B, T = 128, 1000
  env = envs.create(name, batch_size=B, episode_length=T, auto_reset=(name != 'ant'),
                    device=dev)
  zero = torch.zeros((T, B, env.action_size), device=dev)
  st = env.reset(np.array([0, 0], np.uint32))
  st, _ = rollout(env, st, zero)  # warm-up, as the reference's
  torch.cuda.synchronize()
  sps = []
  for seed in range(5):
    st = env.reset(np.array([seed, 0], np.uint32))
    torch.cuda.synchronize()
    t = time.time()
    st, _ = rollout(env, st, zero)
    torch.cuda.synchronize()
    sps.append(B * T / (time.time() - t))
    assert bool(torch.all(st.done != 0))
  assert float(np.mean(sps)) > 1000 * 0.99


@pytest.mark.parametrize('name', ['ant', 'halfcheetah', 'hopper', 'fetch', 'pusher', 'ur5e',
                                  'humanoid', 'grasp'])
def test_rollout_random_equals_slabs_then_rollout(dev, name):
  """bx_env_rollout_random (the actions drawn inside the rollout launch) is
  bit for bit bx_uniform_slabs followed by bx_env_rollout_packed on the
  slabs, and records the same actions; the kinds whose env program reads the
  raw action row are refused, and RolloutRunner falls back to the two
  launches for them."""
  import ctypes as C
  from brax_amd import _native, envs
  from brax_amd.envs.rollout import RolloutRunner, rollout
  B, K = 64, 6
  env = envs.create(name, batch_size=B, episode_length=4, auto_reset=True, device=dev)
  A = env.action_size
  st0 = env.reset(np.array([3, 1], np.uint32))
  seed, off, stride = 5, 1000, 3 * B * A
  runner = RolloutRunner(env, st0, K, seed=seed, offset=off, step_stride=stride)
  assert runner.draw == (name not in ('humanoid', 'grasp'))
  runner.run()
  acts = torch.empty((K, B, A), dtype=torch.float32, device=dev)
  _native.check(_native.lib().bx_uniform_slabs(
      C.c_void_p(acts.data_ptr()), B * A, K, seed, off, stride, None, 0, -1.0, 1.0,
      C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
  final, tr = rollout(env, st0, acts)
  got = runner.trajectory()
  torch.cuda.synchronize()
  assert torch.equal(runner.actions(), acts)
  assert torch.equal(got.qp[..., :13], tr.qp[..., :13])
  assert torch.equal(got.obs, tr.obs) and torch.equal(got.reward, tr.reward)
  assert torch.equal(got.done, tr.done) and torch.equal(got.steps, tr.steps)
  if tr.rng is not None:
    assert torch.equal(got.rng, tr.rng)
  assert torch.equal(runner.state().obs, final.obs)


def test_strided_autoreset_target(dev):
  """An AutoReset target (info['first_qp']) given as four separate
  (B, N, 3|4) tensors instead of the packed layout (the kernels read it
  through its bx_qp strides): the same bits as the packed target, for K-step
  rollouts and single steps."""
  import brax_amd
  from brax_amd import envs
  from brax_amd.envs.rollout import rollout
  env = envs.create('ant', batch_size=64, episode_length=3, auto_reset=True, device=dev)
  st0 = env.reset(np.array([3, 5], np.uint32))
  fq = st0.info['first_qp']
  strided = brax_amd.QP(pos=fq.pos.contiguous(), rot=fq.rot.contiguous(),
                        vel=fq.vel.contiguous(), ang=fq.ang.contiguous())
  st1 = st0.replace(info={**st0.info, 'first_qp': strided})
  g = torch.Generator(device='cpu').manual_seed(6)
  acts = (torch.rand((8, 64, 8), generator=g) * 2 - 1).to(dev)
  fa, ta = rollout(env, st0, acts)
  fb, tb = rollout(env, st1, acts)
  assert float(ta.done.sum()) > 0  # the AutoReset select ran
  # (the packed records' three pad words are never written)
  for x, y in ((ta.qp[..., :13], tb.qp[..., :13]), (ta.obs, tb.obs), (ta.reward, tb.reward),
               (ta.done, tb.done),
               (ta.steps, tb.steps), (ta.metrics, tb.metrics)):
    assert torch.equal(x, y)
  a, b = st0, st1
  for t in range(4):
    a, b = env.step(a, acts[t]), env.step(b, acts[t])
    assert torch.equal(a.qp.pos, b.qp.pos) and torch.equal(a.obs, b.obs)
    assert torch.equal(a.done, b.done)
