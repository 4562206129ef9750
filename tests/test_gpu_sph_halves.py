"""The spherical joint halves (the Humanoid env kernels at 32 lanes per env:
pbd_kernels.hip joint_apply_half_sph / act_torque_half_sph): the partner
exchange on its own, and the 32-lane kernels against the 16-lane kernel they
replace, bit for bit (BX_SPH_HALVES=0 builds a system without them). The
16-lane kernel itself is held to the reference by test_gpu_parity's Humanoid
goldens, which the default (32-lane) env kernels run too.
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


def _same(a, b, t):
  for x, y in ((a.qp.pos, b.qp.pos), (a.qp.rot, b.qp.rot), (a.qp.vel, b.qp.vel),
               (a.qp.ang, b.qp.ang), (a.obs, b.obs), (a.reward, b.reward), (a.done, b.done)):
    assert torch.equal(x, y), (t, float((x - y).abs().max()))


def test_env_lanes(dev):
  """Humanoid's env kernels take the halves; Ant, HalfCheetah and
  HumanoidStandup (its 22 ground rows: two per lane at 16 lanes) do not."""
  from brax_amd import envs
  assert _env('humanoid', 8, True, dev).unwrapped.sys.env_lanes == 32
  assert _env('humanoid', 8, False, dev).unwrapped.sys.env_lanes == 16
  for name in ('ant', 'halfcheetah', 'humanoidstandup'):
    s = envs.create(name, batch_size=8, device=dev).unwrapped.sys
    assert s.env_lanes == s.lanes == 16, name


@pytest.mark.parametrize('B', [1, 255, 4096])
def test_halves_match_the_16_lane_kernel(dev, B):
  """Env.step (one launch per step, Episode + AutoReset: the episodes end
  inside the run) and a K-step rollout launch: every output bit-identical
  to the 16-lane kernel's, at an odd batch (a half-filled last wave) too."""
  from brax_amd.envs.rollout import rollout
  on, off = _env('humanoid', B, True, dev), _env('humanoid', B, False, dev)
  assert on.unwrapped.sys.env_lanes == 32 and off.unwrapped.sys.env_lanes == 16
  a, b = on.reset(np.array([4, 2], np.uint32)), off.reset(np.array([4, 2], np.uint32))
  _same(a, b, 'reset')
  g = torch.Generator(device='cpu').manual_seed(B)
  steps = 12 if B < 4096 else 4
  for t in range(steps):
    act = (torch.rand((B, on.action_size), generator=g) * 2 - 1).to(dev)
    a, b = on.step(a, act), off.step(b, act)
    _same(a, b, t)
  assert B == 4096 or float(a.done.sum()) > 0
  acts = (torch.rand((10, B, on.action_size), generator=g) * 2 - 1).to(dev)
  fa, ta = rollout(on, a, acts)
  fb, tb = rollout(off, b, acts)
  assert torch.equal(ta.qp, tb.qp) and torch.equal(ta.obs, tb.obs)
  assert torch.equal(ta.reward, tb.reward) and torch.equal(ta.done, tb.done)
  _same(fa, fb, 'rollout')
