"""The C restatement (oracle/) pinned to the reference's golden vectors.

Float64 restatement vs the reference's own float64 numpy execution: agreement
to ~1e-10 shows the restatement is the reference's algorithm, so it can check
the HIP path at sizes the goldens do not cover."""
import math

import numpy as np
import pytest

from tests.conftest import golden
from tests.helpers import (CAPSULES, NN_MASKED, SHORT_SCENES, ENVTRAJ_KERNEL, POINTS, ROBOTS, SPRING_ENVS, SPRING_ROBOTS,
                           XCOL, XY_ENVS, env_coef, env_golden, golden_reset_qp, prep_oracle,
                           compiled, env_kind, obs_flags)

ENV_TRAJ = ['ant', 'humanoid', 'halfcheetah', 'humanoidstandup'] + SPRING_ENVS
SYS_TRAJ = (['mountain1', 'mountain2', 'mountain4', 'mountain1nn', 'mountain4nn'] + ROBOTS + CAPSULES + NN_MASKED + POINTS
            + SPRING_ROBOTS + XCOL + SHORT_SCENES)


def _oracle(oracle_lib, name, guard=False, dtype=np.float64):
  vc, d, rd, meta = compiled(name)
  return oracle_lib.Oracle(d, rd, dtype, safe_guard=guard)


@pytest.mark.parametrize('name', ENV_TRAJ + SYS_TRAJ)
def test_system_step_matches_reference(oracle_lib, name):
  o = _oracle(oracle_lib, name)
  T = golden('traj_' + name)
  # float64 rounding-order differences accumulate over a step's substeps:
  # 1e-9 at <= 40 substeps; the CapsuleTest 'ground' scene runs 10000 (a
  # rolling capsule, and Info sums 5000 contact impulses, normwise 10x)
  tol0 = 1e-9 * max(1, int(o.desc['substeps']) // 40)
  rng = np.random.default_rng(0)
  for t in range(T['action'].shape[0]):
    out, info = o.system_step(T['qp'][t], T['action'][t])
    tol = tol0
    if name in ('capsule_capsule_s', 'capsule_cull_s'):
      # states 7-23 steps into a resting stack (contacts chattering at their
      # gates): float64 rounding order differs by up to 6e-9 there
      tol = 1e-8
    if name in XCOL:
      # the extended contact functions select among near-ties (SAT argmax
      # over 576 edge pairs, the closest of 4 segment-triangle candidates):
      # where a rounding-level change of the input flips the choice, float64
      # itself is ill-conditioned there (box_box steps 8-9: 1e-14 relative
      # input noise moves the state 1e-7), so the bound is 4x the state's
      # response to three such perturbations
      q = T['qp'][t]
      cond = max(np.abs(o.system_step(q * (1 + rng.uniform(-1e-14, 1e-14, q.shape)),
                                      T['action'][t])[0] - out).max() for _ in range(3))
      tol = max(tol0, 4 * cond)
    assert np.abs(out - T['qp'][t + 1]).max() < tol
    ic = T['info_contact'][t]
    assert np.abs(info['contact'] - ic).max() < 10 * tol * max(1., np.abs(ic).max())
    ia = T['info_actuator'][t]
    assert np.abs(info['actuator'] - ia).max() < tol * max(1., np.abs(ia).max())
    got, ref = info['contact_penetration'], T['contact_penetration'][t]
    if (np.asarray(o.desc['col_cutoff']) > 0).any():
      # culled Info rows are in top_k order, and exactly tied distances (the
      # symmetric start) are ordered -- and at the cutoff, chosen --
      # arbitrarily by numpy's argpartition/argsort, while the oracle follows
      # jax.lax.top_k (lower index first). Compare the contacts that act
      # (penetration > 0) as multisets; the state check above already pins
      # that the same contacts were applied.
      got, ref = np.sort(np.maximum(got, 0), -1), np.sort(np.maximum(ref, 0), -1)
    pen = np.abs(got - ref)
    assert pen.size == 0 or pen.max() < max(1e-11, tol)


@pytest.mark.parametrize('name', ENV_TRAJ)
def test_contact_info_matches_reference(oracle_lib, name):
  """Info.contact_pos / contact_normal (`_get_contact_info`,
  system.py:36-43) of every Env.step's System.step, row for row."""
  o = _oracle(oracle_lib, name)
  T = golden('traj_' + name)
  for t in range(T['action'].shape[0]):
    _, info = o.system_step(T['qp'][t], T['action'][t])
    for k in ('contact_pos', 'contact_normal'):
      assert info[k].shape == T[k][t].shape, k
      assert np.abs(info[k] - T[k][t]).max() < 1e-9, k


@pytest.mark.parametrize('name', ENV_TRAJ + XY_ENVS + ENVTRAJ_KERNEL)
def test_env_step_matches_reference(oracle_lib, name):
  o = prep_oracle(_oracle(oracle_lib, name), name)
  T = golden(env_golden(name))
  O, M = T['obs'].shape[-1], T['metrics'].shape[-1]
  for t in range(T['action'].shape[0]):
    _, obs, rew, done, met = o.env_step(env_kind(name), T['qp'][t], T['action'][t], O, M,
                                        obs_flags=obs_flags(name), coef=env_coef(name))
    assert np.abs(obs - T['obs'][t + 1]).max() < 1e-9
    assert np.abs(rew - T['reward'][t]).max() < 1e-12
    assert np.array_equal(done, T['done'][t])
    if M:
      assert np.abs(met - T['metrics'][t]).max() < 1e-12


@pytest.mark.parametrize('name', ENV_TRAJ + XY_ENVS + ENVTRAJ_KERNEL)
def test_reset_matches_reference(oracle_lib, name):
  o = _oracle(oracle_lib, name)
  T = golden(env_golden(name))
  qp0 = golden_reset_qp(name, o, T)
  assert np.abs(qp0 - T['qp'][0]).max() < 1e-12
  ic = o.system_info(qp0)
  B = qp0.shape[0]
  obs = o.env_obs(env_kind(name), qp0, ic, np.zeros((B, o.A)), T['obs'].shape[-1],
                  obs_flags=obs_flags(name), coef=env_coef(name))
  assert np.abs(obs - T['reset_obs']).max() < 1e-12


def test_safe_norm_guard_is_negligible(oracle_lib):
  # jit's allclose(x, 0) zero guard (jumpy.py:183-189) vs the numpy path
  T = golden('traj_ant')
  a = _oracle(oracle_lib, 'ant', guard=True).system_step(T['qp'][3], T['action'][3])[0]
  b = _oracle(oracle_lib, 'ant', guard=False).system_step(T['qp'][3], T['action'][3])[0]
  assert np.abs(a - b).max() < 1e-7


def test_fp32_envelope(oracle_lib):
  """Brax's algorithm in fp32 stays within SURVEY §8(c)'s envelope."""
  T = golden('traj_ant')
  o = _oracle(oracle_lib, 'ant', guard=True, dtype=np.float32)
  out, _ = o.system_step(T['qp'][2], T['action'][2])
  ref = T['qp'][3]
  nw = lambda a, b: (np.abs(a - b).max(axis=(1, 2)) / np.maximum(1, np.abs(b).max(axis=(1, 2))))
  assert nw(out[..., 0:3], ref[..., 0:3]).max() < 1e-5
  assert nw(out[..., 7:10], ref[..., 7:10]).max() < 1e-3


def test_closest_segment_kats(oracle_lib):
  o = _oracle(oracle_lib, 'ant')
  k = golden('kat')
  a, b = o.closest_segments(k['seg_in'])
  assert np.abs(a - k['seg_a']).max() < 1e-12 and np.abs(b - k['seg_b']).max() < 1e-12
  # the reference's own literal cases (geometry_test.py:217-272)
  cases = [
      ([[0.73432405, 0.12372768, 0.20272314], [1.10600128, 0.88555209, 0.65209485],
        [0.85599262, 0.61736299, 0.9843583], [1.84270939, 0.92891793, 1.36343326]],
       [1.09063, 0.85404, 0.63351], [0.99596, 0.66156, 1.03813], 5),
      ([[0, 0, -1], [0, 0, 1], [-1, 0, 0], [1, 0, 0]], [0, 0, 0], [0, 0, 0], 5),
      ([[0.2, 0.2, 0], [1, 1, 0], [0.2, 0.4, 0], [1, 2, 0]], [0.3, 0.3, 0], [0.2, 0.4, 0], 2),
      ([[0, 0, -1], [0, 0, 1], [1, 0, -1], [1, 0, 1]], [0, 0, 0], [1, 0, 0], 5),
      ([[0, 0, -1], [0, 0, 1], [1, 0, 1], [1, 0, 3]], [0, 0, 1], [1, 0, 1], 5),
      ([[0, 0, -1], [0, 0, -1], [1, 0, 0.1], [1, 0, 0.1]], [0, 0, -1], [1, 0, 0.1], 5),
      ([[0, 0, -1], [0, 0, 1], [0, 0, -1], [0, 0, 1]], [0, 0, 0], [0, 0, 0], 5),
  ]
  for seg, ea, eb, places in cases:
    a, b = o.closest_segments(np.array(seg, np.float64))
    np.testing.assert_allclose(a[0], ea, atol=1.5 * 10**-places)
    np.testing.assert_allclose(b[0], eb, atol=1.5 * 10**-places)


@pytest.mark.parametrize('name', ['wrap_ant', 'wrap_ant_ar2'])
def test_wrapper_semantics(oracle_lib, name):
  """Episode + AutoReset semantics (wrappers.py:105-148) restated in numpy on
  top of the oracle's unwrapped env step, vs the reference's wrapped rollout;
  wrap_ant_ar2: action_repeat 2 (the EpisodeWrapper scans two env steps per
  step and sums their rewards; steps advance by 2)."""
  T = golden(name)
  o = _oracle(oracle_lib, 'ant')
  ep = int(T['episode_length'])
  ar = int(T['action_repeat']) if 'action_repeat' in T else 1
  qp, obs = T['qp'][0], T['obs'][0]
  done = T['done'][0]
  steps = T['steps'][0]
  for t in range(T['action'].shape[0]):
    steps = np.where(done != 0, 0.0, steps)
    q, rew = qp, 0.0
    for _ in range(ar):
      q, obs1, r, d_in, _ = o.env_step('ant', q, T['action'][t], 87, 10)
      rew = rew + r
    qp1 = q
    steps = steps + ar
    done = np.where(steps >= ep, 1.0, d_in)
    trunc = np.where(steps >= ep, 1 - d_in, 0.0)
    sel = done != 0
    qp = np.where(sel[:, None, None], T['first_qp'], qp1)
    obs = np.where(sel[:, None], T['first_obs'], obs1)
    assert np.abs(qp - T['qp'][t + 1]).max() < 1e-9
    assert np.abs(obs - T['obs'][t + 1]).max() < 1e-9
    assert np.abs(rew - T['reward'][t + 1]).max() < 1e-12
    assert np.array_equal(done, T['done'][t + 1])
    assert np.array_equal(steps, T['steps'][t + 1])
    assert np.array_equal(trunc, T['truncation'][t + 1])


@pytest.mark.parametrize('target', [15., 30., 45., 90.])
def test_spring_1d_actuator_float64(oracle_lib, target):
  """Actuator1DTest (`physics_legacy_test.py:555-594`) as the reference runs
  it (numpy float64): the diverging spring joint sends the bob to |pos| ~
  1e84 while its unit rotation holds the target angle (2 places)."""
  from brax_amd import compiler
  from tests.test_gpu_spring_kat import ACT1, _cfg
  vc, d, meta = compiler.compile_system(_cfg(ACT1))
  o = oracle_lib.Oracle(d, compiler.compile_reset(vc, meta['body_index']), np.float64)
  out, _ = o.system_step(o.default_qp(np.zeros((1, 1)), np.zeros((1, 1))), np.array([[target]]))
  assert np.abs(out[0, 1, 0:3]).max() > 1e80
  # Revolute.axis_angle (joints.py:311-319) about the joint's x axis: the
  # rotation is about x alone, so the angle is 2 atan2(q_x, q_w) mod 2 pi
  w, x = out[0, 1, 3], out[0, 1, 4]
  ang = math.remainder(2 * math.atan2(x, w), 2 * math.pi)
  assert round(abs(target * math.pi / 180 - ang), 2) == 0


def test_force_kats_float64(oracle_lib):
  """The reference's ForceTest (`physics_test.py:813-831`) holds for the
  float64 restatement, as for the reference's own (numpy, float64) run."""
  from brax_amd import compiler
  from brax_amd import config as cfgmod
  text = """
    dt: 0.1 substeps: 5000
    bodies { name: "body" mass: 1 inertia { x: 1 y: 1 z: 1 } }
    forces { name: "thruster" body: "body" strength: 2.5 thruster {} }
    forces { name: "twister" body: "body" strength: 2.5 twister {} }"""
  vc, d, meta = compiler.compile_system(cfgmod.parse(text))
  o = oracle_lib.Oracle(d, compiler.compile_reset(vc, meta['body_index']), np.float64)
  qp = np.zeros((1, 1, 13))
  qp[..., 3] = 1
  for f in (1, 5, 10):
    out, _ = o.system_step(qp, f * np.array([[1., 0, 0, 0, 0, 0]]))
    assert round(abs(out[0, 0, 0] - 0.5 * 2.5 * f * 0.1 ** 2), 3) == 0
    out, _ = o.system_step(qp, f * np.array([[0, 0, 0, 1., 0, 0]]))
    assert round(abs(out[0, 0, 10] - 2.5 * f * 0.1), 3) == 0
