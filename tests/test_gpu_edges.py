"""Edge cases of the batch axis and of the boundary, on the GPU.

* Ragged batches: a batch that leaves the last workgroup part-empty (SINGLE
  mode packs 4 envs per wavefront, the item loops 64 / L) steps every env to
  the bits it has inside a full batch — for the SINGLE-mode kernel, the
  item-loop kernel and the MULTI-mode kernel.
* Empty batches: reset and step of 0 envs return empty tensors (the
  reference's vmap over an empty axis) and launch nothing.
* A scene past one workgroup's LDS is refused at construction with the
  reason, not run.
"""
import numpy as np
import pytest
import torch

from tests.helpers import config_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _batch_rows(qp, rows):
  import brax_amd
  return brax_amd.QP(*(getattr(qp, f)[rows].contiguous() for f in ('pos', 'rot', 'vel', 'ang')))


def _same(a, b):
  for f in ('pos', 'rot', 'vel', 'ang'):
    assert torch.equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize('B', [1, 3, 5, 63, 65])
def test_env_step_ragged_batch(dev, B):
  """Ant Env.step (SINGLE mode, 4 envs per wavefront): env e of a ragged
  batch of B steps to the bits of env e of a full batch of 68."""
  from brax_amd import envs
  env = envs.create('ant', batch_size=68, episode_length=1000, auto_reset=True, device=dev)
  full = env.reset(np.array([3, 9], np.uint32))
  act = torch.rand((68, env.action_size), device=dev, generator=torch.Generator(dev).manual_seed(B)) * 2 - 1
  nfull = env.step(full, act)
  rows = torch.arange(B, device=dev)
  part = full.replace(qp=_batch_rows(full.qp, rows), obs=full.obs[:B], reward=full.reward[:B],
                      done=full.done[:B], metrics={k: v[:B] for k, v in full.metrics.items()},
                      info={k: (v[:B] if torch.is_tensor(v) and v.dim() >= 1 and v.shape[0] == 68
                                else (_batch_rows(v, rows) if k == 'first_qp' else v))
                            for k, v in full.info.items()})
  npart = env.step(part, act[:B].contiguous())
  torch.cuda.synchronize()
  _same(npart.qp, _batch_rows(nfull.qp, rows))
  assert torch.equal(npart.obs, nfull.obs[:B])
  assert torch.equal(npart.reward, nfull.reward[:B])
  assert torch.equal(npart.done, nfull.done[:B])


@pytest.mark.parametrize('name,B', [('ant', 7), ('capsule_cull', 3), ('mountain2', 3)])
def test_system_step_ragged_batch(dev, name, B):
  """System.step on the SINGLE-mode (ant), item-loop (capsule_cull: culled,
  not SINGLE) and MULTI-mode (mountain2) kernels: a ragged batch steps to the
  bits of the same envs in a larger batch."""
  import brax_amd
  s = brax_amd.System(config_for(name), device=dev)
  n = 20
  qp0 = s.default_qp()
  g = torch.Generator(dev).manual_seed(11)
  big = brax_amd.QP(*(t.unsqueeze(0).expand((n,) + t.shape).contiguous()
                      for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))
  big = big.replace(vel=big.vel + 0.1 * torch.randn(big.vel.shape, device=dev, generator=g))
  A = max(s.action_size, 1)
  act = torch.rand((n, A), device=dev, generator=g) * 2 - 1
  if s.action_size == 0:
    act = act[:, :0]
  qf, _ = s.step(big, act)
  rows = torch.arange(B, device=dev)
  qb, _ = s.step(_batch_rows(big, rows), act[:B].contiguous())
  torch.cuda.synchronize()
  _same(qb, _batch_rows(qf, rows))


def test_empty_batch(dev):
  """0 envs: reset and step return empty tensors of the right trailing
  shapes."""
  from brax_amd import envs
  env = envs.get_environment('ant', device=dev)
  st = env.reset_batch(np.array([0, 1], np.uint32), 0)
  assert st.qp.pos.shape == (0, env.sys.num_bodies, 3) and st.obs.shape == (0, env.observation_size)
  nst = env.step(st, torch.zeros((0, env.action_size), device=dev))
  torch.cuda.synchronize()
  assert nst.qp.pos.shape[0] == 0 and nst.obs.shape == (0, env.observation_size)
  assert nst.reward.shape == (0,) and nst.done.shape == (0,)
  qp, info = env.sys.step(nst.qp, torch.zeros((0, env.action_size), device=dev))
  assert qp.pos.shape[0] == 0 and info.contact_penetration.shape[0] == 0


def test_scene_past_lds_is_refused(dev):
  """Ant Mountain(32) (32 ants, 289 bodies, ~45k capsule pairs) does not fit
  one workgroup's LDS: construction raises with the reason."""
  import brax_amd
  from brax_amd._native import NativeError
  from brax_amd.envs.mountain import ant_mountain_config
  with pytest.raises((NativeError, ValueError), match='LDS|too many|large'):
    brax_amd.System(ant_mountain_config(32), device=dev)


@pytest.mark.parametrize('name,cutoff', [('ant', 0), ('humanoid', 0), ('mountain4', 0),
                                         ('mountain4', 36), ('capsule_cull', 0)])
def test_step_without_info_is_the_same_state(dev, name, cutoff):
  """`System.step(qp, act, info=False)` (no Info outputs: the large-scene
  kernel also skips far capsule pairs on its last collision pass, whose rows
  only feed Info) steps to the bits of the full step, for the SINGLE,
  item-loop and MULTI kernels."""
  import brax_amd
  cfg = config_for(name)
  if cutoff:
    cfg.collider_cutoff = cutoff
  sys_ = brax_amd.System(cfg, device=dev)
  B = 64
  q0 = sys_.default_qp()
  qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                     for t in (q0.pos, q0.rot, q0.vel, q0.ang)))
  g = torch.Generator(dev).manual_seed(4)
  for _ in range(3):
    act = torch.rand((B, max(sys_.action_size, 1)), device=dev, generator=g) * 2 - 1
    a, info = sys_.step(qp, act)
    b, none = sys_.step(qp, act, info=False)
    assert info is not None and none is None
    _same(a, b)
    qp = a
  # mid-trajectory: the golden rollout's last state per env, each copy's
  # positions / velocities perturbed, so capsule pairs cross the broad
  # phase's reach (in both directions) on the last collision pass, the one
  # info=False also culls
  from tests.conftest import golden
  T = golden('traj_' + name)['qp'][-1]
  rng = np.random.default_rng(5)
  q = np.repeat(T, (B + T.shape[0] - 1) // T.shape[0], axis=0)[:B].copy()
  q[..., 0:3] += rng.uniform(-0.02, 0.02, q[..., 0:3].shape)
  q[..., 7:10] += rng.uniform(-0.5, 0.5, q[..., 7:10].shape)
  q[..., 10:13] += rng.uniform(-1.0, 1.0, q[..., 10:13].shape)
  from brax_amd.base import qp_from_numpy
  qp = qp_from_numpy(q, dev)
  for _ in range(6):
    act = torch.rand((B, max(sys_.action_size, 1)), device=dev, generator=g) * 2 - 1
    a, _ = sys_.step(qp, act)
    b, _ = sys_.step(qp, act, info=False)
    _same(a, b)
    qp = a
