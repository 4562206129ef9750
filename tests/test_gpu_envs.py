"""The torch env layer over the other registered envs vs the reference's own
rollouts (tests/golden/envtraj_*: `env.reset` from seeds, random actions,
`env.step`, numpy backend, float64).

Two checks per env and step:
  * the env layer alone: `_get_obs` / `_step` of the golden post-step state
    (fp32 evaluation of the reference's formulas) against the golden obs,
    reward, done and metrics, normwise <= 2e-5;
  * the whole `Env.step` (fused physics kernel + env layer) from the golden
    state: the new state within the fp32 envelope of Brax's algorithm (as in
    test_gpu_parity), obs and reward finite and within 2e-3 normwise (they
    carry the state's fp32 error, amplified by 1/dt for velocities).
"""
import numpy as np
import pytest
import torch

from tests.conftest import golden
from tests.helpers import QP_FIELDS, normwise

pytestmark = pytest.mark.gpu

ENVS = ['grasp']
TOL = 2e-5


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _state(env, T, t, dev):
  from brax_amd.base import qp_from_numpy
  from brax_amd.envs.env import State
  qp = qp_from_numpy(T['qp'][t], dev)
  B = T['qp'].shape[1]
  keys = [str(k) for k in T['metric_keys']]
  met = {k: torch.zeros((B,), device=dev) for k in keys}
  if t > 0:
    for i, k in enumerate(keys):
      met[k] = torch.as_tensor(T['metrics'][t - 1][:, i], dtype=torch.float32, device=dev)
  obs = torch.as_tensor(T['obs'][t], dtype=torch.float32, device=dev)
  z = torch.zeros((B,), device=dev)
  return State(qp=qp, obs=obs, reward=z, done=z.clone(), metrics=met, info={})


def _info(T, t, dev, which='info_contact'):
  """brax Info of the golden step t (only contact.vel is read by env layers)."""
  from brax_amd.base import Info, P
  c = torch.as_tensor(T[which][t], dtype=torch.float32, device=dev)
  return Info(contact=P(c[..., :3], c[..., 3:]), joint=None, actuator=None, contact_pos=None,
              contact_normal=None, contact_penetration=None)


def _close(got, ref, tol, what):
  got = np.asarray(got, np.float64)
  ref = np.asarray(ref, np.float64)
  assert np.all(np.isfinite(got)), what
  nw = normwise(got.reshape(got.shape[0], -1), ref.reshape(ref.shape[0], -1))
  assert nw.max() <= tol, f'{what}: normwise {nw.max():.3e} > {tol:.1e}'


@pytest.mark.parametrize('name', ENVS)
def test_env_layer_vs_golden(dev, name):
  from brax_amd import envs
  from brax_amd.base import qp_from_numpy
  env = envs.get_environment(name, device=dev)
  T = golden('envtraj_' + name)
  keys = [str(k) for k in T['metric_keys']]
  # reset observation of the golden reset state
  if name not in ('ur5e', 'grasp', 'fetch'):  # their reset obs read the reset-time Info
    _close(env._get_obs(qp_from_numpy(T['qp'][0], dev), None).cpu(), T['reset_obs'], TOL,
           'reset obs')
  for t in range(T['action'].shape[0]):
    st = _state(env, T, t, dev)
    act = torch.as_tensor(T['action'][t], dtype=torch.float32, device=dev)
    q1 = T['qp'][t + 1].copy()
    if hasattr(env, '_teleport'):
      # obs and reward are taken before a hit target is teleported (grasp.py:
      # 150-183, ur5e.py:60-88); the target body does not move in the physics
      q1[:, env.target_idx] = T['qp'][t][:, env.target_idx]
    new = env._step(st, act, qp_from_numpy(q1, dev), _info(T, t, dev))
    _close(new.obs.cpu(), T['obs'][t + 1], TOL, f'obs t={t}')
    _close(new.reward.cpu()[:, None], T['reward'][t][:, None], TOL, f'reward t={t}')
    assert np.array_equal(new.done.cpu().numpy(), T['done'][t]), f'done t={t}'
    for i, k in enumerate(keys):
      _close(new.metrics[k].cpu()[:, None], T['metrics'][t][:, i:i + 1], TOL, f'{k} t={t}')


@pytest.mark.parametrize('name', ENVS)
def test_env_step_vs_golden(dev, oracle_lib, name):
  from brax_amd import envs
  from tests.helpers import compiled
  env = envs.get_environment(name, device=dev)
  T = golden('envtraj_' + name)
  _, d, rd, _ = compiled(name)
  o32s = [oracle_lib.Oracle(d, rd, np.float32, safe_guard=True, fma=f) for f in (False, True)]
  o64 = oracle_lib.Oracle(d, rd, np.float64)
  for t in range(T['action'].shape[0]):
    st = _state(env, T, t, dev)
    act = torch.as_tensor(T['action'][t], dtype=torch.float32, device=dev)
    new = env.step(st, act)
    # the (qp, action) the env fed to the kernel (swimmer adds drag forces,
    # grasp moves the palm first)
    qp_in, sys_act = env._pre_step(st, env._action(act, act.shape[0]))
    qp_in, sys_act = qp_in.numpy(), sys_act.cpu().numpy()
    ref, _ = o64.system_step(qp_in, sys_act)
    rng = np.random.default_rng(1234)
    ins = [qp_in] + [qp_in * (1 + rng.uniform(-6e-8, 6e-8, qp_in.shape)) for _ in range(3)]
    outs = [o.system_step(q.astype(np.float32), sys_act.astype(np.float32))[0]
            for o in o32s for q in ins]
    got = new.qp.numpy()
    if hasattr(env, '_teleport'):  # teleported targets draw from the device RNG
      got[:, env.target_idx] = ref[:, env.target_idx]
    for f, sl in QP_FIELDS.items():
      e32 = np.max([normwise(x[..., sl], ref[..., sl]) for x in outs])
      nw = normwise(got[..., sl], ref[..., sl])
      assert nw.max() <= max(1e-5, 2 * e32), f'{f} t={t}: {nw.max():.3e} vs e32 {e32:.3e}'
    # the golden's next state came from float64 actions incl. float64 drag
    _close(new.obs.cpu(), T['obs'][t + 1], 2e-3, f'obs t={t}')
    _close(new.reward.cpu()[:, None], T['reward'][t][:, None], 2e-3, f'reward t={t}')


@pytest.mark.parametrize('name', ['grasp'])
def test_wrapped_torch_env(dev, name):
  """Episode + AutoReset over a torch env run as device tensor ops."""
  from brax_amd import envs
  env = envs.create(name, batch_size=16, episode_length=5, auto_reset=True, device=dev)
  st = env.reset(np.array([3, 1], np.uint32))
  A = env.action_size
  for k in range(12):
    st = env.step(st, torch.rand((16, A), device=dev) * 2 - 1)
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


@pytest.mark.parametrize('name', ['ur5e', 'fetch'])
def test_target_teleport_stream(dev, name):
  """The target envs' hit-target teleport (ur5e.py:107-113, fetch.py:93-99):
  a target placed on the torso is hit, moves onto the ring [radius, radius +
  distance) at the target height, and every env's stream advances by one per
  step; reruns are bit-identical. (The reference draws from JAX keys: the
  spot itself is parity-unpinned.)"""
  from brax_amd import envs
  env = envs.get_environment(name, device=dev)
  B = 64
  st = env.reset_batch(np.array([5, 9], np.uint32), B)
  rng0 = st.info['rng'].clone()
  t, g = int(env.coef[0]), int(env.coef[1])
  act = torch.zeros((B, env.action_size), device=dev)
  # half the envs get their target where the torso will be after the step
  # (the target takes no part in the physics)
  ahead = env.step(st, act).qp.pos[:, t]
  pos = st.qp.pos.clone()
  pos[:B // 2, g] = ahead[:B // 2]
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
  radius, distance, height = env.ring
  assert (r >= radius - 1e-4).all() and (r <= radius + distance + 1e-4).all()
  np.testing.assert_allclose(tg[:B // 2, 2], height, atol=1e-6)
  # targets that were not hit stay where the physics left them
  np.testing.assert_array_equal(tg[B // 2:], st.qp.pos[B // 2:, g].cpu().numpy())
  assert len(set(map(tuple, np.round(tg[:B // 2], 5)))) == B // 2  # distinct spots
