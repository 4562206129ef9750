"""The spherical joint halves (opt-in, BX_SPH_HALVES=1: the Humanoid env
kernels at 32 lanes per env, pbd_kernels.hip joint_apply_half_sph /
act_torque_half_sph; measured slower than the default 16-lane kernel): the
partner exchange on its own, and the 32-lane kernels' K-step rollout launch
bit for bit against their own chained steps. Their results against the
reference's goldens: test_gpu_parity.py test_env_step_vs_golden[humanoid:sph]
(the same gate as the 16-lane kernel's; the two kernels are not bit-identical).
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


@pytest.mark.parametrize('lanes', [16, 32])
def test_partner_exchange(dev, lanes):
  """Lane l receives lane l ^ lanes / 2's value (DPP row rotation at 16
  lanes, v_permlane16_swap at 32)."""
  from brax_amd import _native
  out = torch.full((64,), -1.0, device=dev)
  stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
  _native.check(_native.lib().bx_debug_partner(C.c_void_p(out.data_ptr()), lanes, stream))
  torch.cuda.synchronize()
  want = (np.arange(64) ^ (lanes // 2)).astype(np.float32)
  np.testing.assert_array_equal(out.cpu().numpy(), want)


def _env(name, B, halves, dev):
  from brax_amd import envs
  old = os.environ.get('BX_SPH_HALVES')
  os.environ['BX_SPH_HALVES'] = '1' if halves else '0'
  try:
    return envs.create(name, batch_size=B, episode_length=7, auto_reset=True, device=dev)
  finally:
    if old is None:
      del os.environ['BX_SPH_HALVES']
    else:
      os.environ['BX_SPH_HALVES'] = old


def test_env_lanes(dev):
  """Humanoid's env kernels take the halves when asked; by default, and for
  Ant, HalfCheetah and HumanoidStandup (its 22 ground rows: two per lane at
  16 lanes) never."""
  from brax_amd import envs
  assert _env('humanoid', 8, True, dev).unwrapped.sys.env_lanes == 32
  assert _env('humanoid', 8, False, dev).unwrapped.sys.env_lanes == 16
  assert envs.create('humanoid', batch_size=8, device=dev).unwrapped.sys.env_lanes == 16
  for name in ('ant', 'halfcheetah', 'humanoidstandup'):
    s = envs.create(name, batch_size=8, device=dev).unwrapped.sys
    assert s.env_lanes == s.lanes == 16, name


@pytest.mark.parametrize('B', [1, 255, 4096])
def test_halves_rollout_matches_their_steps(dev, B):
  """The halves' K-step rollout launch bit for bit against their own chained
  Env.step launches (Episode + AutoReset: the 7-step episodes end inside the
  run), at an odd batch (a half-filled last wave) too. Their parity with the
  reference: test_gpu_parity's test_env_step_vs_golden[humanoid:sph]."""
  from brax_amd.envs.rollout import rollout
  on = _env('humanoid', B, True, dev)
  assert on.unwrapped.sys.env_lanes == 32
  st0 = on.reset(np.array([4, 2], np.uint32))
  g = torch.Generator(device='cpu').manual_seed(B)
  acts = (torch.rand((10, B, on.action_size), generator=g) * 2 - 1).to(dev)
  final, tr = rollout(on, st0, acts)
  st = st0
  for t in range(acts.shape[0]):
    st = on.step(st, acts[t])
    q = torch.cat([st.qp.pos, st.qp.rot, st.qp.vel, st.qp.ang], -1)
    assert torch.equal(tr.qp[t][..., :13], q), t
    assert torch.equal(tr.obs[t], st.obs) and torch.equal(tr.reward[t], st.reward), t
    assert torch.equal(tr.done[t], st.done), t
  assert float(tr.done.sum()) > 0  # the episodes ended inside the rollout
  assert torch.equal(final.qp.pos, st.qp.pos) and torch.equal(final.obs, st.obs)
