"""Standalone SoA phase kernels vs the float64 oracle's phases."""
import numpy as np
import pytest
import torch

from tests.conftest import golden
from tests.helpers import QP_FIELDS, compiled, normwise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def setup(oracle_lib):
  import brax_amd
  from tests.helpers import config_for
  dev = torch.device('cuda', 0)
  sys_ = brax_amd.System(config_for('ant'), device=dev)
  _, d, rd, _ = compiled('ant')
  return sys_, oracle_lib.Oracle(d, rd, np.float64), dev


def _soa(a, dev):
  return torch.as_tensor(a, dtype=torch.float32).permute(2, 1, 0).contiguous().to(dev)


def _aos(t):
  return t.permute(2, 1, 0).double().cpu().numpy()


def test_kinetic(setup):
  from brax_amd import phases
  sys_, o, dev = setup
  qp = golden('traj_ant')['qp'][2]
  got = _aos(phases.kinetic(sys_, _soa(qp, dev)))
  ref = o.phase(0, qp)
  for f, sl in QP_FIELDS.items():
    assert normwise(got[..., sl], ref[..., sl]).max() < 2e-6, f


def test_update_acc(setup):
  from brax_amd import phases
  sys_, o, dev = setup
  qp = golden('traj_ant')['qp'][3]
  dp = np.random.default_rng(0).normal(size=qp.shape[:2] + (6,))
  got = _aos(phases.update_acc(sys_, _soa(qp, dev), _soa(dp, dev)))
  ref = o.phase(1, qp, dp)
  assert normwise(got, ref).max() < 2e-6


def test_velocity_projection(setup):
  from brax_amd import phases
  sys_, o, dev = setup
  T = golden('traj_ant')
  prev, qp = T['qp'][1], o.phase(0, T['qp'][1])  # one kinetic step apart
  got = _aos(phases.velocity_projection(sys_, _soa(qp, dev), _soa(prev, dev)))
  ref = o.phase(2, qp, prev)
  for f, sl in QP_FIELDS.items():
    # velocities are position differences / h: fp32 input rounding x 1/h
    tol = 2e-6 if f in ('pos', 'rot') else 5e-4
    assert normwise(got[..., sl], ref[..., sl]).max() < tol, f


def test_capsule_plane(setup):
  from brax_amd import phases
  sys_, o, dev = setup
  qp = golden('traj_ant')['qp'][4]
  got = phases.capsule_plane(sys_, _soa(qp, dev)).permute(2, 1, 0).double().cpu().numpy()
  ref = o.capsule_plane(qp)
  assert normwise(got, ref).max() < 2e-6


def test_large_batch_roundtrip(setup):
  """B = 65536 envs: SoA kinetic matches the fused-kernel layout conversion
  (to_soa/from_soa) and stays finite."""
  from brax_amd import phases
  sys_, o, dev = setup
  qp = golden('traj_ant')['qp'][5]
  B = 65536
  big = np.tile(qp, (B // qp.shape[0], 1, 1))
  soa = _soa(big, dev)
  out = phases.kinetic(sys_, soa)
  got = _aos(out)
  ref = o.phase(0, qp)
  assert np.isfinite(got).all()
  assert normwise(got[:64], ref).max() < 2e-6
  assert normwise(got[-64:], ref).max() < 2e-6
