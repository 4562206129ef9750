"""System compiler vs the reference's own compiled arrays (tests/golden/desc_*)."""
import numpy as np
import pytest

from brax_amd import compiler
from tests.conftest import golden
from tests.helpers import ROBOTS, compiled, config_for

NAMES = ['ant', 'humanoid', 'halfcheetah', 'mountain1', 'mountain2', 'mountain4'] + ROBOTS


@pytest.mark.parametrize('name', NAMES)
def test_descriptor_bit_exact(name):
  _, d, _, _ = compiled(name)
  g = golden('desc_' + name)
  for k in g.files:
    a, b = np.asarray(d[k]), g[k]
    assert a.shape == b.shape, k
    # integer index arrays bit-exact; float constants computed in the same
    # float64 operation order -> bit-exact too
    assert np.array_equal(a, b), k


def test_ant_structure():
  _, d, rd, meta = compiled('ant')
  assert meta['action_size'] == 8 and int(d['n_bodies']) == 10
  assert len(d['row_group']) == 5 and d['col_oneway'].tolist() == [1]
  # ground (body 9) is frozen: a OneWay plane, masks zero
  assert d['pos_mask'][9].sum() == 0 and d['quat_mask'][9].tolist() == [1, 0, 0, 0]
  # reset: one lifted tree (torso + 8 legs), ground separate
  assert rd['n_root_groups'] == 2
  assert (rd['body_root_group'][:9] == rd['body_root_group'][0]).all()


def test_humanoid_sphericalized():
  vc, d, rd, meta = compiled('humanoid')
  # App. A.2: mixed dofs -> one Spherical group, act_index padded with -1
  assert set(d['joint_type'].tolist()) == {3}
  assert d['joint_free_dofs'].tolist() == [2, 1, 3, 1, 3, 1, 2, 1, 2, 1]
  assert (d['act_index'] == -1).sum() == 30 - 17
  assert meta['num_joint_dof'] == 17


def test_parents_generator_quirk():
  # App. A.1: parent/child pairs are NOT excluded (generator consumed early)
  _, d, _, _ = compiled('mountain1')
  pairs = set(zip(d['row_body_a'][d['row_group'] == 1].tolist(),
                  d['row_body_b'][d['row_group'] == 1].tolist()))
  assert (0, 1) in pairs or (1, 0) in pairs


def test_unsupported_raise():
  cfg = config_for('ant')
  cfg.collider_cutoff = 3
  cfg2 = config_for('mountain2')
  cfg2.collider_cutoff = 3
  with pytest.raises(NotImplementedError):
    compiler.compile_system(cfg2)
  cfg3 = config_for('ant')
  cfg3.dynamics_mode = 'legacy_spring'
  with pytest.raises(ValueError):
    compiler.compile_system(cfg3)


def test_default_angle_matches_reference_reset():
  vc, d, rd, meta = compiled('ant')
  T = golden('traj_ant')
  da = compiler.default_angle(vc)
  # reset_qpos = default_angle + U[-0.1, 0.1] noise
  assert np.all(np.abs(T['reset_qpos'] - da[None]) <= 0.1 + 1e-12)
