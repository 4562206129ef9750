"""The revolute joint halves' partner exchange on its own (bx_debug_partner):
the DPP row rotation that hands each side lane of an Ant / HalfCheetah joint
its partner side's values (pbd_kernels.hip `xh`, joint_apply_half). The
round-4 opt-in 32-lane spherical halves measured slower than the 16-lane
kernel (Humanoid rollout 37.7 vs 32.1 us per step) and were removed (ABI 13)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def test_partner_exchange(dev):
  """Lane l receives lane l ^ 8's value within each env of 16 lanes."""
  from brax_amd import _native
  out = torch.full((64,), -1.0, device=dev)
  stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
  _native.check(_native.lib().bx_debug_partner(C.c_void_p(out.data_ptr()), 16, stream))
  torch.cuda.synchronize()
  want = (np.arange(64) ^ 8).astype(np.float32)
  np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_partner_exchange_refuses_other_widths(dev):
  from brax_amd import _native
  out = torch.full((64,), -1.0, device=dev)
  assert _native.lib().bx_debug_partner(C.c_void_p(out.data_ptr()), 32, None) != 0
