"""Env-layer behaviour on the device beyond the per-kind golden parity of
test_gpu_parity: wrappers (Episode / AutoReset fused in the step kernel,
EvalWrapper, gym), wrapped rollouts of every kernel env kind, and the target
envs' teleport streams.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


@pytest.mark.parametrize('name', ['hopper', 'walker2d', 'inverted_pendulum',
                                  'inverted_double_pendulum', 'acrobot', 'reacher',
                                  'reacherangle', 'swimmer', 'pusher', 'ur5e', 'fetch', 'grasp'])
def test_wrapped_kernel_env(dev, name):
  """Episode + AutoReset over each kernel env kind: one launch per step,
  finite states, step counters within the episode length, and bit-identical
  reruns from the same state."""
  from brax_amd import envs
  env = envs.create(name, batch_size=16, episode_length=5, auto_reset=True, device=dev)
  st = env.reset(np.array([3, 1], np.uint32))
  A = env.action_size
  g = torch.Generator(device=dev).manual_seed(7)
  for _ in range(12):
    act = torch.rand((16, A), device=dev, generator=g) * 2 - 1
    nxt = env.step(st, act)
    again = env.step(st, act)
    assert torch.equal(nxt.qp.pos, again.qp.pos) and torch.equal(nxt.obs, again.obs)
    st = nxt
    assert torch.isfinite(st.obs).all() and torch.isfinite(st.qp.pos).all()
    assert int(st.info['steps'].max()) <= 5
  assert 'truncation' in st.info and 'first_qp' in st.info


def test_eval_wrapper_accumulates(dev):
  """EvalWrapper (`wrappers.py:169-203`): episode metrics are the sums of the
  per-step metrics while the episode is active; steps freeze when done."""
  from brax_amd import envs
  env = envs.create('ant', batch_size=32, episode_length=4, eval_metrics=True, device=dev)
  st = env.reset(np.array([0, 11], np.uint32))
  em0 = st.info['eval_metrics']
  assert float(em0.active_episodes.min()) == 1.0
  sums = torch.zeros(32, device=dev)
  active = torch.ones(32, device=dev)
  for k in range(6):
    st = env.step(st, torch.rand((32, 8), device=dev) * 2 - 1)
    sums = sums + st.reward * active
    active = active * (1 - st.done)
  em = st.info['eval_metrics']
  torch.testing.assert_close(em.episode_metrics['reward'], sums)
  torch.testing.assert_close(em.active_episodes, active)
  assert float(em.episode_steps.max()) <= 4


def test_vector_gym_wrapper(dev):
  """VectorGymWrapper / create_gym_env (`wrappers.py:265-337`,
  `envs/__init__.py:118-130`): device tensors out, auto-reset inside."""
  from brax_amd import envs
  from brax_amd.envs.to_torch import JaxToTorchWrapper
  g = JaxToTorchWrapper(envs.create_gym_env('ant', batch_size=64, seed=3, device=dev),
                        device=dev)
  obs = g.reset()
  assert obs.shape == (64, 87) and obs.is_cuda
  assert g.action_space.shape == (64, 8) and g.single_observation_space.shape == (87,)
  for _ in range(3):
    obs, reward, done, info = g.step(torch.rand((64, 8), device=dev) * 2 - 1)
  assert reward.shape == (64,) and done.shape == (64,)
  assert 'truncation' in info and 'x_velocity' in info
  single = envs.create_gym_env('hopper', device=dev)
  o = single.reset()
  assert o.shape[-1] == single.observation_space.shape[0]


@pytest.mark.parametrize('name', ['ur5e', 'fetch', 'grasp'])
def test_target_teleport_stream(dev, name):
  """The target envs' hit-target teleport (ur5e.py:107-113, fetch.py:93-99,
  grasp.py:119-125): a target placed where the torso (grasp: the object)
  will be is hit, moves onto the ring [radius, radius + distance) at the
  target height (grasp: a height in [0, 8)), and every env's stream advances
  by one per step; reruns are bit-identical. (The reference draws from JAX
  keys: the spot itself is parity-unpinned.)"""
  from brax_amd import envs
  env = envs.get_environment(name, device=dev)
  B = 64
  st = env.reset_batch(np.array([5, 9], np.uint32), B)
  rng0 = st.info['rng'].clone()
  c = env.coef
  if name == 'grasp':
    t, g, radius, distance, height = int(c[1]), int(c[2]), c[4], c[5], None
  else:
    t, g, radius, distance, height = int(c[0]), int(c[1]), c[2], c[3], c[4]
  act = torch.zeros((B, env.action_size), device=dev)
  # half the envs get their target where the torso will be after the step,
  # the others far away
  # (the target takes no part in the physics)
  ahead = env.step(st, act).qp.pos[:, t]
  pos = st.qp.pos.clone()
  pos[:B // 2, g] = ahead[:B // 2]
  pos[B // 2:, g] = ahead[B // 2:] + torch.tensor([40., 0., 0.], device=dev)  # out of reach
  from brax_amd.base import QP
  st = st.replace(qp=QP(pos=pos, rot=st.qp.rot, vel=st.qp.vel, ang=st.qp.ang))
  a = env.step(st, act)
  b = env.step(st, act)
  assert torch.equal(a.qp.pos, b.qp.pos) and torch.equal(a.obs, b.obs)
  assert torch.equal(a.info['rng'], rng0 + 1)
  hit = a.metrics['hits'].cpu().numpy()
  assert hit[:B // 2].all() and not hit[B // 2:].any()
  tg = a.qp.pos[:, g].cpu().numpy()
  r = np.linalg.norm(tg[:B // 2, :2], axis=-1)
  assert (r >= radius - 1e-4).all() and (r <= radius + distance + 1e-4).all()
  if height is None:
    assert (tg[:B // 2, 2] >= 0).all() and (tg[:B // 2, 2] < 8).all()
  else:
    np.testing.assert_allclose(tg[:B // 2, 2], height, atol=1e-6)
  # targets that were not hit stay where the physics left them
  np.testing.assert_array_equal(tg[B // 2:], st.qp.pos[B // 2:, g].cpu().numpy())
  assert len(set(map(tuple, np.round(tg[:B // 2], 5)))) == B // 2  # distinct spots


@pytest.mark.parametrize('name', ['reacher', 'reacherangle', 'pusher', 'ur5e', 'fetch', 'grasp'])
def test_body_placing_reset_is_one_call(dev, name):
  """`bx_env_reset` places the bodies these envs' resets place (reacher.py:
  156-174, reacherangle.py:44-60, pusher.py:178-209, ur5e.py:41-58,
  fetch.py:41-57, grasp.py:54-70) and starts the target envs' streams, in
  the one C call: its state equals the explicit path (`reset_draws`: the
  same counter draws at the same indices, placements formed on the host in
  float64, then `reset_from`), the noise bit for bit."""
  import ctypes as C
  from brax_amd import abi, _native
  from brax_amd.envs import tasks
  from brax_amd.envs import env as env_mod
  from brax_amd.system import _stream
  from brax_amd import envs
  env = envs.get_environment(name, device=dev)
  B, off = 48, 100
  key = np.array([3, 17], np.uint32)
  st = env.reset_batch(key, B, env_offset=off)
  if name == 'grasp':
    D = env.sys.num_joint_dof
    ref = env.reset_from(env.sys.default_angle().reshape(1, -1).expand(B, -1),
                         torch.zeros((B, D), device=dev))
  else:
    ref = env.reset_from(**env.reset_draws(key, B, env_offset=off))
  torch.cuda.synchronize()
  for f in ('pos', 'rot', 'vel', 'ang'):
    a, b = getattr(st.qp, f), getattr(ref.qp, f)
    assert torch.allclose(a, b, atol=2e-6, rtol=1e-6), (f, float((a - b).abs().max()))
  # the joint noise is the same draw, bit for bit: every body the reset does
  # not place (the joint tree's, from the same angles through the same
  # default_qp kernel) is bit-identical; only the placements, formed on the
  # host in float64 on the explicit path, may differ by rounding
  from tests.helpers import reset_bodies
  placed = {env.sys._body_index[b] for b in reset_bodies(name)}  # pylint: disable=protected-access
  assert placed or name == 'grasp'
  keep = [b for b in range(env.sys.num_bodies) if b not in placed]
  for f in ('pos', 'rot', 'vel', 'ang'):
    a, b = getattr(st.qp, f)[:, keep], getattr(ref.qp, f)[:, keep]
    assert torch.equal(a, b), (f, float((a - b).abs().max()))
  assert torch.allclose(st.obs, ref.obs, atol=1e-5, rtol=1e-5)
  assert float(st.reward.abs().max()) == 0 and float(st.done.abs().max()) == 0
  if getattr(env, 'needs_rng', False):
    want = tasks.rng_streams(env_mod.key_to_seed(key), off, B, dev)
    assert torch.equal(st.info['rng'], want)
    # the C ABI refuses a target env reset without the stream buffer
    out = abi.BxEnvState()
    qp, obs, scal, met = env._alloc(B)
    out.qp = env_mod.qp_struct(qp, True)
    out.obs, out.reward, out.done = obs.data_ptr(), scal.data_ptr(), scal.data_ptr() + 4 * B
    out.metrics = met.data_ptr()
    p = env._params()
    rc = _native.lib().bx_env_reset(env.sys._h, C.byref(p), B, 1, 0, None, 0.1, C.byref(out),
                                    _stream(dev.index))
    assert rc != 0 and b'rng' in _native.lib().bx_last_error()


@pytest.mark.parametrize('name', ['ant', 'reacher', 'pusher', 'ur5e', 'grasp'])
def test_vmap_reset_uses_each_envs_key(dev, name):
  """`VmapWrapper.reset` over a (B, 2) key batch (wrappers.py:79-80): env e
  depends on key e only (its draws and, for the target envs, its stream),
  equals a one-env reset from that key, and a repeated key repeats the env."""
  from brax_amd import envs
  from brax_amd.envs import wrappers
  env = envs.get_environment(name, device=dev)
  keys = np.stack([np.array([i, 3 * i + 1], np.uint32) for i in range(16)])
  st = wrappers.VmapWrapper(env).reset(keys)
  assert st.qp.pos.shape[0] == 16
  for e in (0, 5, 15):
    one = wrappers.VmapWrapper(env).reset(keys[e:e + 1])
    assert torch.equal(one.qp.pos[0], st.qp.pos[e]) and torch.equal(one.obs[0], st.obs[e])
    if 'rng' in st.info:
      assert torch.equal(one.info['rng'][0], st.info['rng'][e])
  keys2 = keys.copy()
  keys2[3] = keys2[9]
  st2 = wrappers.VmapWrapper(env).reset(keys2)
  assert torch.equal(st2.qp.pos[3], st2.qp.pos[9]) and torch.equal(st2.obs[3], st2.obs[9])
  if name != 'grasp':  # grasp's reset draws nothing but its stream
    assert not torch.equal(st.qp.pos[3], st.qp.pos[9])
  if 'rng' in st.info:
    assert torch.equal(st2.info['rng'][3], st2.info['rng'][9])
    assert not torch.equal(st.info['rng'][3], st.info['rng'][9])
