"""System compiler vs the reference's own compiled arrays (tests/golden/desc_*)."""
import numpy as np
import pytest

from brax_amd import compiler
from tests.conftest import golden
from tests.helpers import (CAPSULES, NN_MASKED, POINTS, ROBOTS, SPRING_ENVS, SPRING_ROBOTS, XCOL, compiled,
                           config_for)

NAMES = (['ant', 'humanoid', 'halfcheetah', 'humanoidstandup', 'mountain1', 'mountain2', 'mountain4', 'mountain1nn', 'mountain4nn']
         + ROBOTS + CAPSULES + NN_MASKED + POINTS + SPRING_ENVS + SPRING_ROBOTS + XCOL)


@pytest.mark.parametrize('name', NAMES)
def test_descriptor_bit_exact(name):
  _, d, _, _ = compiled(name)
  g = golden('desc_' + name)
  # every descriptor field is pinned: the reference dump holds exactly the
  # compiler's keys
  assert set(g.files) == set(d.keys()), sorted(set(g.files) ^ set(d.keys()))
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


def test_spring_groups():
  """legacy_spring (spring_joints.py:302-331): joints grouped by dof without
  sphericalisation -> Revolute, Universal, Spherical groups; actuators index
  every dof (no -1 padding); spring defaults from stiffness."""
  _, d, _, meta = compiled('humanoid_spring')
  assert int(d['dynamics_mode']) == compiler.DYN_LEGACY_SPRING
  assert sorted(set(d['joint_type'].tolist())) == [1, 2, 3]
  assert (np.diff(d['joint_group']) >= 0).all() and (d['joint_free_dofs'] == -1).all()
  assert meta['num_joint_dof'] == 17 and (d['act_index'] >= 0).sum() == 17
  assert (d['joint_stiffness'] > 0).all() and (d['joint_limit_strength'] > 0).all()


def test_unsupported_raise():
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


def test_near_neighbors_cells():
  """NearNeighbors (colliders.py:55-89, 1005-1013): candidate rows are the
  allowed cells of the U x U candidate matrix, addressed by BODY index; cells
  outside U x U are dropped as jit's scatter drops them."""
  cfg = config_for('mountain2')
  cfg.collider_cutoff = 18
  _, d, _ = compiler.compile_system(cfg)
  g = int(np.flatnonzero(d['col_cutoff'])[0])
  rows = d['row_group'] == g
  flat = d['row_flat'][rows]
  assert (np.diff(flat) > 0).all() and d['col_cutoff'][g] == 18
  U = 18  # unique capsule candidates of two ants
  i, j = flat // U, flat % U
  assert (i < U).all() and (j < U).all() and (i != j).all()
  # Ant 1's bodies sit at 10..18 (after the ground): cells on body 18 drop
  assert not ((d['row_body_a'][rows] == 18) | (d['row_body_b'][rows] == 18)).all()
  # ant without cutoff: every group is Pairs
  _, d0, _ = compiler.compile_system(config_for('ant'))
  assert (d0['col_cutoff'] == 0).all() and (d0['row_flat'] == -1).all()
  # more cutoff than allowed cells (still < the 153 pairs: culled): top_k's
  # tail is the masked cells of lowest flat index, flagged
  n = int(rows.sum())
  cfg.collider_cutoff = n + 3
  _, d2, _ = compiler.compile_system(cfg)
  rows2 = d2['row_group'] == g
  m = d2['row_nn_masked'][rows2]
  assert m.sum() == 3 and rows2.sum() == n + 3
  flat2 = d2['row_flat'][rows2]
  assert (np.diff(flat2) > 0).all()
  allowed = set(flat.tolist())
  masked = [f for f in range(U * U) if f not in allowed][:3]
  assert sorted(flat2[m == 1].tolist()) == masked
  # a cutoff at or past the pairs is no culling at all (colliders.py:1003-1005)
  cfg.collider_cutoff = 153
  _, d3, _ = compiler.compile_system(cfg)
  assert (d3['col_cutoff'] == 0).all()
