"""The spherical joint halves (opt-in, BX_SPH_HALVES=1: the Humanoid env
kernels at 32 lanes per env, pbd_kernels.hip joint_apply_half_sph /
act_torque_half_sph; measured slower than the default 16-lane kernel): the
partner exchange on its own, the 32-lane kernels' K-step rollout launch bit
for bit against their own chained steps, and both against the 16-lane kernel
(which test_gpu_parity holds to the reference's goldens) within rounding:
the two compile the same arithmetic to differently contracted FMAs (the
first steps from reset differ by ~4e-9).
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


def _close(a, b, t, tol):
  """Every field within `tol` relative to its magnitude; done flags equal."""
  for x, y in ((a.qp.pos, b.qp.pos), (a.qp.rot, b.qp.rot), (a.qp.vel, b.qp.vel),
               (a.qp.ang, b.qp.ang), (a.obs, b.obs), (a.reward, b.reward)):
    err = float((x - y).abs().max() / y.abs().max().clamp(min=1.0))
    assert err <= tol, (t, err)
  assert torch.equal(a.done, b.done), t


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
def test_halves_match_the_16_lane_kernel(dev, B):
  """Env.step (one launch per step, Episode + AutoReset: the episodes end
  inside the run) against the 16-lane kernel within rounding, at an odd batch
  (a half-filled last wave) too; then a K-step rollout launch of the halves
  bit for bit against their own chained Env.step launches."""
  from brax_amd.envs.rollout import rollout
  on, off = _env('humanoid', B, True, dev), _env('humanoid', B, False, dev)
  assert on.unwrapped.sys.env_lanes == 32 and off.unwrapped.sys.env_lanes == 16
  a, b = on.reset(np.array([4, 2], np.uint32)), off.reset(np.array([4, 2], np.uint32))
  _close(a, b, 'reset', 0.0)
  g = torch.Generator(device='cpu').manual_seed(B)
  for t in range(6):  # (the episodes are 7 steps: none ends here)
    act = (torch.rand((B, on.action_size), generator=g) * 2 - 1).to(dev)
    a, b = on.step(a, act), off.step(b, act)
    _close(a, b, t, 1e-5)
  acts = (torch.rand((10, B, on.action_size), generator=g) * 2 - 1).to(dev)
  final, tr = rollout(on, a, acts)
  st = a
  for t in range(acts.shape[0]):
    st = on.step(st, acts[t])
    q = torch.cat([st.qp.pos, st.qp.rot, st.qp.vel, st.qp.ang], -1)
    assert torch.equal(tr.qp[t][..., :13], q), t
    assert torch.equal(tr.obs[t], st.obs) and torch.equal(tr.reward[t], st.reward), t
    assert torch.equal(tr.done[t], st.done), t
  assert float(tr.done.sum()) > 0  # the episodes ended inside the rollout
  assert torch.equal(final.qp.pos, st.qp.pos) and torch.equal(final.obs, st.obs)
