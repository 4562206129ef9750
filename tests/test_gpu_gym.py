"""The gym / torch path against the reference's own:
`JaxToTorchWrapper(create_gym_env('ant', batch_size=8, episode_length=3))`
stepped through the C-ABI vs the golden `gym_ant` that
`oracle/gen_golden.py:gym_ant` records from the reference's VectorGymWrapper
(`wrappers.py:311-314`: obs, reward, done and info = {**state.metrics,
**state.info}, every leaf, every step). Every step starts from the
reference's wrapped state before it (after reset: the reset key itself is
parity-unpinned, threefry being absent offline). Episode length 3 puts truncation, the done-driven
AutoReset select and the step-counter reset inside the 6 steps.

Gates: the per-env envelope gate of tests/test_gpu_parity.py on obs, qp,
reward and every metric leaf (66 fp32 realisations of Brax's algorithm on the
golden's state before the step, with the AutoReset select applied); done,
steps and truncation exactly; first_qp / first_obs exactly the stored reset
state."""
import numpy as np
import pytest
import torch

from tests.conftest import golden
from tests.helpers import QP_FIELDS
from tests.test_gpu_parity import Envelope, _env_err, _gate

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _qp(a, dev):
  from brax_amd.base import qp_from_numpy
  return qp_from_numpy(a, dev)


def test_vector_gym_step_vs_reference(dev, oracle_lib):
  from brax_amd import envs
  from brax_amd.envs.env import State
  from brax_amd.envs.to_torch import JaxToTorchWrapper
  T = golden('gym_ant')
  B, L = T['qp0'].shape[0], int(T['episode_length'])
  g = JaxToTorchWrapper(envs.create_gym_env('ant', batch_size=B, seed=5, episode_length=L,
                                            device=dev), device=dev)
  assert g.num_envs == B and g.action_space.shape == (B, 8)
  assert g.single_observation_space.shape == (87,)
  f32 = lambda a: torch.as_tensor(a, dtype=torch.float32, device=dev)  # noqa: E731

  def wrapped_state(t):
    """The reference's wrapped state before step t: after reset (t = 0) or
    after its step t - 1 (each step then starts from the reference's own
    state: the gym path's reward is (x1 - x0) / dt, which would amplify a
    chained fp32 drift of the state 20x)."""
    if t == 0:
      q, o, r, d, st, tr = (T['qp0'], T['obs0'], T['reward0'], T['done0'], T['steps0'],
                            T['truncation0'])
    else:
      q, o, r, d = T['qp'][t - 1], T['obs'][t - 1], T['reward'][t - 1], T['done'][t - 1]
      st, tr = T['info_steps'][t - 1], T['info_truncation'][t - 1]
    return State(qp=_qp(q, dev), obs=f32(o), reward=f32(r), done=f32(d), metrics={},
                 info={'first_qp': _qp(T['first_qp'], dev), 'first_obs': f32(T['first_obs']),
                       'steps': f32(st), 'truncation': f32(tr)})
  inner = g.env._env.unwrapped  # pylint: disable=protected-access
  keys = [str(k) for k in T['info_keys']]
  mkeys = list(inner.metric_keys)
  assert sorted(mkeys) == sorted(k for k in keys
                                 if k not in ('first_qp', 'first_obs', 'steps', 'truncation'))
  env32 = Envelope(oracle_lib, 'ant')
  for t in range(T['action'].shape[0]):
    g.env._state = wrapped_state(t)  # pylint: disable=protected-access
    # numpy actions in (the gym caller's), converted by the wrapper's action()
    obs, reward, done, info = g.step(T['action'][t].astype(np.float32))
    torch.cuda.synchronize()
    assert sorted(info) == keys, sorted(info)
    for leaf in (obs, reward, done, *(v for k, v in info.items() if k != 'first_qp')):
      assert isinstance(leaf, torch.Tensor) and leaf.device == dev
    before = T['qp0'] if t == 0 else T['qp'][t - 1]
    outs = env32.env('ant', before, T['action'][t], 87, len(mkeys), 0, inner.coef)
    sel = T['done'][t] != 0  # AutoReset: done envs restart from the stored first state
    assert np.array_equal(done.cpu().numpy(), T['done'][t])
    assert np.array_equal(info['steps'].cpu().numpy(), T['info_steps'][t])
    assert np.array_equal(info['truncation'].cpu().numpy(), T['info_truncation'][t])
    e_obs = [np.where(sel[:, None], T['first_obs'], o[1]) for o in outs]
    _gate(obs.cpu().numpy(), T['obs'][t], _env_err(e_obs, T['obs'][t]), 'obs')
    got = g.env._state.qp.numpy()  # pylint: disable=protected-access
    for f, sl in QP_FIELDS.items():
      e_qp = [np.where(sel[:, None, None], T['first_qp'], o[0])[..., sl] for o in outs]
      _gate(got[..., sl], T['qp'][t][..., sl], _env_err(e_qp, T['qp'][t][..., sl]), f)
    _gate(reward.cpu().numpy()[:, None], T['reward'][t][:, None],
          _env_err([o[2][:, None] for o in outs], T['reward'][t][:, None]), 'reward')
    for i, k in enumerate(mkeys):
      ref = T['info_' + k][t][:, None]
      _gate(info[k].cpu().numpy()[:, None], ref, _env_err([o[4][:, i:i + 1] for o in outs], ref), k)
    # the stored reset state rides along unchanged
    np.testing.assert_array_equal(info['first_obs'].cpu().numpy(),
                                  T['first_obs'].astype(np.float32))
    fq = info['first_qp']
    np.testing.assert_array_equal(
        np.concatenate([fq.pos.cpu().numpy(), fq.rot.cpu().numpy(), fq.vel.cpu().numpy(),
                        fq.ang.cpu().numpy()], -1), T['info_first_qp'][t].astype(np.float32))


def test_torch_wrapper_moves_leaves_and_takes_numpy_actions(dev):
  """JaxToTorchWrapper's conversions (`to_torch.py:40-64`): numpy and torch
  actions in, every output leaf on the requested device (here the CPU)."""
  from brax_amd import envs
  from brax_amd.envs.to_torch import JaxToTorchWrapper
  g = JaxToTorchWrapper(envs.create_gym_env('ant', batch_size=4, seed=1, device=dev),
                        device=torch.device('cpu'))
  obs = g.reset()
  assert obs.device.type == 'cpu' and obs.shape == (4, 87)
  obs, reward, done, info = g.step(np.zeros((4, 8), np.float32))
  obs2, _, _, info2 = g.step(torch.zeros((4, 8)))
  assert obs.device.type == 'cpu' and reward.device.type == 'cpu' and done.device.type == 'cpu'
  assert info['first_qp'].pos.device.type == 'cpu'
  assert all(v.device.type == 'cpu' for k, v in info2.items() if k != 'first_qp')
