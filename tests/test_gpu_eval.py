"""EvalWrapper against the reference's own (`wrappers.py:168-202`). Needs an
MI355X.

`tests/golden/eval_ant.npz` (`oracle/gen_golden.py:eval_ant`) is the
reference's `envs.create('ant', episode_length=3, batch_size=8,
eval_metrics=True)` stepped 7 times from its reset (env 3 lifted out of the
healthy range, so it terminates on the first step): every step's state and
`eval_metrics`. The build's chain starts from the golden's reset state (the
reset key is threefry, parity-unpinned) and must give:

* active_episodes and episode_steps exactly (flag and counter work);
* each env's episode metrics (the metrics summed while its first episode is
  active) within its own bound: the sum over its active steps of that step's
  per-env bound max(2e-4, 2 x E32), E32 the fp32 error of Brax's algorithm on
  the step (the oracle's plain and FMA float32 builds on the golden's input
  state and 3 ulp-perturbed copies), normwise as the parity gates;
* done / steps exactly, the state as `test_wrapped_rollout_vs_golden`.
"""
import numpy as np
import pytest
import torch

from tests.conftest import golden
from tests.helpers import compiled, normwise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def test_eval_wrapper_vs_golden(dev, oracle_lib):
  from brax_amd import envs
  from brax_amd.base import qp_from_numpy
  from brax_amd.envs.env import State
  from brax_amd.envs.wrappers import EvalMetrics
  T = golden('eval_ant')
  B = T['qp0'].shape[0]
  keys = [str(k) for k in T['metric_keys']]
  env = envs.create('ant', episode_length=int(T['episode_length']), batch_size=B,
                    eval_metrics=True, device=dev)
  f32 = lambda a: torch.as_tensor(a, dtype=torch.float32, device=dev)  # noqa: E731
  rm = T['reset_metrics']
  em = EvalMetrics(episode_metrics={k: torch.zeros(B, device=dev) for k in keys},
                   active_episodes=torch.ones(B, device=dev),
                   episode_steps=torch.zeros(B, device=dev))
  st = State(qp=qp_from_numpy(T['qp0'], dev), obs=f32(T['obs0']),
             reward=torch.zeros(B, device=dev), done=torch.zeros(B, device=dev),
             metrics={k: f32(rm[:, i]) for i, k in enumerate(keys) if k != 'reward'},
             info={'first_qp': qp_from_numpy(T['first_qp'], dev), 'first_obs': f32(T['first_obs']),
                   'steps': torch.zeros(B, device=dev), 'truncation': torch.zeros(B, device=dev),
                   'eval_metrics': em})
  _, d, rd, _ = compiled('ant')
  os32 = [oracle_lib.Oracle(d, rd, np.float32, fma=f) for f in (False, True)]
  ant_keys = sorted(k for k in keys if k != 'reward')
  rng = np.random.default_rng(5)
  bound = np.zeros(B)
  active = np.ones(B)
  q_in = T['qp0']
  for t in range(T['action'].shape[0]):
    st = env.step(st, f32(T['action'][t]))
    em = st.info['eval_metrics']
    assert sorted(em.episode_metrics) == keys
    # the step's per-env fp32 envelope of every metric, from the golden's input
    ref_m = None
    e32 = np.zeros(B)
    with np.errstate(all='ignore'):
      o64 = oracle_lib.Oracle(d, rd, np.float64)
      _, _, r64, _, m64 = o64.env_step('ant', q_in, T['action'][t], 87, 10)
      ref_m = np.concatenate([m64, r64[:, None]], -1)
      for o in os32:
        for k in range(4):
          q = (q_in * (1 + (rng.uniform(-6e-8, 6e-8, q_in.shape) if k else 0))).astype(np.float32)
          _, _, r32, _, m32 = o.env_step('ant', q, T['action'][t].astype(np.float32), 87, 10)
          e32 = np.maximum(e32, normwise(np.concatenate([m32, r32[:, None]], -1), ref_m))
    bound += active * np.maximum(2e-4, 2 * e32)
    active = T['active_episodes'][t]
    got = np.stack([em.episode_metrics[k].cpu().numpy() for k in keys], -1)
    nw = normwise(got, T['episode_metrics'][t])
    assert (nw <= np.maximum(bound, 1e-5)).all(), (t + 1, nw, bound)
    assert np.array_equal(em.active_episodes.cpu().numpy(), T['active_episodes'][t]), t + 1
    assert np.array_equal(em.episode_steps.cpu().numpy(), T['episode_steps'][t]), t + 1
    assert np.array_equal(st.done.cpu().numpy(), T['done'][t]), t + 1
    assert np.array_equal(st.info['steps'].cpu().numpy(), T['steps'][t]), t + 1
    for f, sl in (('pos', slice(0, 3)), ('rot', slice(3, 7))):
      assert normwise(st.qp.numpy()[..., sl], T['qp'][t][..., sl]).max() <= 1e-4, (t + 1, f)
    q_in = T['qp'][t]
  assert ant_keys == sorted(env.metric_keys)
