"""The reference's physics scenario tests (`brax/tests/physics_test.py`), run
through the HIP kernels with the reference's own expected outcomes and
tolerances (assertAlmostEqual places). SURVEY §8(c) "pins to port as KATs".

The scene descriptions are the tests' config text, kept here as input data.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _sys(text, dev, **over):
  import brax_amd
  from brax_amd import config as cfgmod
  cfg = cfgmod.parse(text)
  for k, v in over.items():
    setattr(cfg, k, v)
  return brax_amd.System(cfg, device=dev)


def _qp(pos, rot, vel, ang, dev):
  from brax_amd.base import QP
  t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)  # noqa: E731
  return QP(pos=t(pos), rot=t(rot), vel=t(vel), ang=t(ang))


def places(a, b, n):
  """unittest assertAlmostEqual(a, b, places=n)."""
  assert round(abs(float(a) - float(b)), n) == 0, (float(a), float(b), n)


SPHERE = """
dt: 5 substeps: 500 friction: 0.6 gravity { z: -9.8 }
bodies { name: "Sphere1" mass: 1 colliders { sphere { radius: 0.25 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Ground" frozen { all: true } colliders { plane {} } }
defaults { qps { name: "Sphere1" pos { z: 1 } } }
defaults { qps { name: "Sphere1" pos { z: 1 } vel { x: 2 } } }
"""


def test_sphere_hits_ground(dev):
  """`physics_test.py:275-280`."""
  s = _sys(SPHERE, dev)
  qp, _ = s.step(s.default_qp(0), torch.zeros(0, device=dev))
  places(qp.pos[0, 2], 0.25, 2)


def test_sphere_roll(dev):
  """`physics_test.py:282-287`: default 1 starts with vel x = 2 (set here
  explicitly: the device reset compiles defaults index 0)."""
  s = _sys(SPHERE, dev)
  qp = _qp([[0, 0, 1], [0, 0, 0]], [[1, 0, 0, 0]] * 2, [[2, 0, 0], [0, 0, 0]], [[0, 0, 0]] * 2,
           dev)
  qp, _ = s.step(qp, torch.zeros(0, device=dev))
  assert float(qp.ang[0, 1]) > 0.25


JOINT = """
substeps: 4000 dt: .01 gravity { z: -9.8 }
bodies { name: "Anchor" frozen { all: true } mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Bob" mass: 1 inertia { x: 1 y: 1 z: 1 } }
joints { name: "Joint" parent: "Anchor" child: "Bob" child_offset { z: 1 }
         angle_limit { min: -180 max: 180 } }
solver_scale_pos: .2
"""


@pytest.mark.parametrize('mass,radius,vel', [(2.0, 0.125, 0.0625), (5.0, 0.125, 0.03125),
                                             (1.0, 0.0625, 0.1)])
def test_pendulum_period(dev, mass, radius, vel):
  """`physics_test.py:497-523`: a small-angle pendulum returns to the origin
  after one period."""
  import brax_amd
  from brax_amd import config as cfgmod
  cfg = cfgmod.parse(JOINT)
  cfg.dt = 2 * math.pi * math.sqrt((.4 * radius ** 2 + 1.) / 9.8)
  cfg.bodies[1].mass = mass
  for ax in 'xyz':
    setattr(cfg.bodies[1].inertia, ax, .4 * mass * radius ** 2)
  s = brax_amd.System(cfg, device=dev)
  qp = _qp([[0., 0., 0.], [0., 0., -1.]], [[1., 0., 0., 0.]] * 2, [[0., 0., 0.], [0., vel, 0.]],
           [[0., 0., 0.], [vel, 0., 0.]], dev)
  qp, _ = s.step(qp, torch.zeros(0, device=dev))
  places(qp.pos[1, 1], 0., 3)


ACT1 = """
substeps: 80 dt: 4.0
bodies { name: "Anchor" frozen { all: true } mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Bob" mass: 1 inertia { x: 1 y: 1 z: 1 } }
joints { name: "Joint" parent: "Anchor" child: "Bob" child_offset { z: 1 }
         angle_limit { min: -180 max: 180 } angular_damping: 20.0 }
actuators { name: "Joint" joint: "Joint" strength: 150.0 angle {} }
defaults { qps { name: "Anchor" pos { z: 2 } } qps { name: "Bob" pos { z: 1 } } }
"""


@pytest.mark.parametrize('target', [15., 30., 45., 90.])
def test_1d_angle_actuator(dev, target):
  """`physics_test.py:624-636`."""
  s = _sys(ACT1, dev)
  qp, _ = s.step(s.default_qp(), torch.tensor([target], device=dev))
  angle, _ = s.joints[0].angle_vel(qp)
  places(target * math.pi / 180, angle[0], 2)


ACT2 = """
substeps: 2000 dt: 2.0
bodies { name: "Anchor" frozen { all: true } mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Bob" mass: 1 inertia { x: 1 y: 1 z: 1 } }
joints { name: "Joint" parent: "Anchor" child: "Bob" child_offset { z: 1 }
         angle_limit { min: -180 max: 180 } angle_limit { min: -180 max: 180 }
         angular_damping: 20.0 }
actuators { name: "Joint" joint: "Joint" strength: 200.0 angle {} }
defaults { qps { name: "Anchor" pos { z: 2 } } qps { name: "Bob" pos { z: 1 } } }
"""


@pytest.mark.parametrize('t1,t2', [(15., 30.), (-45., 80), (120, -60.), (-35., -52.)])
def test_2d_angle_actuator(dev, t1, t2):
  """`physics_test.py:668-679`: a 2-dof joint, sphericalised."""
  s = _sys(ACT2, dev)
  qp, _ = s.step(s.default_qp(), torch.tensor([t1, t2], device=dev))
  angles, _ = s.joints[0].angle_vel(qp)
  places(t1 * math.pi / 180, angles[0], 2)
  places(t2 * math.pi / 180, angles[1], 2)


ACT3 = """
substeps: 8000 dt: 20
bodies { name: "Anchor" frozen { all: true } mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Bob" mass: 1 inertia { x: 1 y: 1 z: 1 } colliders { capsule { radius: 0.5 length: 2.0 } } }
joints { name: "Joint" parent: "Anchor" child: "Bob" child_offset { z: 1 }
         angle_limit { min: -100 max: 100 } angle_limit { min: -100 max: 100 }
         angle_limit { min: -100 max: 100 } angular_damping: 180.0 }
actuators { name: "Joint" joint: "Joint" strength: 40.0 torque {} }
defaults { qps { name: "Anchor" pos { z: 2 } } qps { name: "Bob" pos { z: 1 } } }
"""


@pytest.mark.parametrize('limits', [(15, 15, 15), (35, 40, 75), (80, 45, 30)])
def test_3d_torque_actuator(dev, limits):
  """`physics_test.py:724-742`: torque drives each dof to its limit."""
  import brax_amd
  from brax_amd import config as cfgmod
  for t in [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1)]:
    cfg = cfgmod.parse(ACT3)
    for al, lim in zip(cfg.joints[0].angle_limit, limits):
      al.min, al.max = -lim, lim
    s = brax_amd.System(cfg, device=dev)
    qp, _ = s.step(s.default_qp(), torch.tensor(t, dtype=torch.float32, device=dev))
    angles, _ = s.joints[0].angle_vel(qp)
    for a, lim, tq in zip(angles.tolist(), limits, t):
      if tq != 0:
        places(a * 180 / math.pi, lim, 1)


FORCE = """
dt: 0.1 substeps: 5000
bodies { name: "body" mass: 1 inertia { x: 1 y: 1 z: 1 } }
forces { name: "thruster" body: "body" strength: 2.5 thruster {} }
forces { name: "twister" body: "body" strength: 2.5 twister {} }
"""


def _fp32_budget(oracle_lib, text, act_dir, field, want_per_unit):
  """The reference runs these two tests un-jitted, i.e. numpy float64, with
  h = 2e-5 s over 5000 substeps. In fp32 the velocity projection's
  q * q_prev^-1 cancellation makes Brax's own algorithm miss the expected
  value by up to ~4 % (the oracle's float32 build: 3.9 % for the unit
  twister), systematically rather than randomly, and the HIP path's
  reciprocal-based division lands elsewhere in the same band. The GPU is
  held to 1.5x the worst relative fp32 miss over the test's three
  magnitudes; test_oracle holds the float64 restatement to the reference's
  own 3-decimal tolerance."""
  from brax_amd import compiler
  from brax_amd import config as cfgmod
  vc, d, meta = compiler.compile_system(cfgmod.parse(text))
  o = oracle_lib.Oracle(d, compiler.compile_reset(vc, meta['body_index']), np.float32)
  qp = np.zeros((1, 1, 13))
  qp[..., 3] = 1
  rel = 0.
  for m in (1, 5, 10):
    out, _ = o.system_step(qp, (m * np.asarray(act_dir, np.float64))[None])
    rel = max(rel, abs(float(out[0, 0, field]) / (m * want_per_unit) - 1))
  return 1.5 * rel


@pytest.mark.parametrize('force', [1, 5, 10])
def test_thruster(dev, oracle_lib, force):
  """`physics_test.py:813-821`."""
  s = _sys(FORCE, dev)
  a = force * np.array([1., 0., 0., 0., 0., 0])
  qp, _ = s.step(s.default_qp(), torch.tensor(a, dtype=torch.float32, device=dev))
  want = 0.5 * 2.5 * force * 0.1 ** 2
  err = abs(float(qp.pos[0][0]) - want)
  budget = _fp32_budget(oracle_lib, FORCE, [1., 0, 0, 0, 0, 0], 0, 0.5 * 2.5 * 0.1 ** 2)
  assert err <= max(5e-4, budget * want), (err, budget)


@pytest.mark.parametrize('torque', [1, 5, 10])
def test_twister(dev, oracle_lib, torque):
  """`physics_test.py:823-831`."""
  s = _sys(FORCE, dev)
  a = torque * np.array([0., 0., 0., 1., 0., 0])
  qp, _ = s.step(s.default_qp(), torch.tensor(a, dtype=torch.float32, device=dev))
  want = 2.5 * torque * 0.1
  err = abs(float(qp.ang[0][0]) - want)
  budget = _fp32_budget(oracle_lib, FORCE, [0, 0, 0, 1., 0, 0], 10, 2.5 * 0.1)
  assert err <= max(5e-4, budget * want), (err, budget)


SPHERICALIZE = """
substeps: 2 dt: .01 gravity { z: 0.0 }
bodies { name: "Segment_1" mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Segment_2" mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Segment_3" mass: 1 inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Segment_4" mass: 1 inertia { x: 1 y: 1 z: 1 } }
joints { name: "Joint_1_2" parent: "Segment_1" child: "Segment_2" child_offset { z: 1 }
         angle_limit { min: -180 max: 180 } }
joints { name: "Joint_2_3" parent: "Segment_2" child: "Segment_3" child_offset { z: 1 }
         angle_limit { min: -180 max: 180 } angle_limit { min: -180 max: 180 } }
joints { name: "Joint_3_4" parent: "Segment_3" child: "Segment_4" child_offset { z: 1 }
         angle_limit { min: -180 max: 180 } angle_limit { min: -180 max: 180 }
         angle_limit { min: -180 max: 180 } }
"""


def test_sphericalize_free_dofs(dev):
  """`physics_test.py:775-790`: one spherical group, free dofs [1, 2, 3]."""
  s = _sys(SPHERICALIZE, dev)
  assert len(s.joints) == 1
  assert list(s.joints[0].free_dofs) == [1, 2, 3]
  a, v = s.joints[0].angle_vel(s.default_qp())
  assert a.shape == (6,) and v.shape == (6,)


ELASTIC = """
dt: 0.01 substeps: 10 friction: 0.0 elasticity: 1.0 gravity { z: -9.8 }
bodies { name: "sphere" mass: 1 colliders { capsule { radius: .5 length: 1.0 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "sphere_stationary" mass: 1 colliders { capsule { radius: .5 length: 1.0 } }
         inertia { x: 1 y: 1 z: 1 } }
bodies { name: "boxwall" mass: 1 colliders { box { halfsize { x: 1 y: 1 z: 1 } } }
         inertia { x: 1 y: 1 z: 1 } frozen { all: true } }
bodies { name: "Ground" frozen { all: true } colliders { plane {} } }
defaults { qps { name: "sphere" vel { x: 10 y: 0 z: 0 } pos { z: .5 } }
           qps { name: "sphere_stationary" pos { x: -20 y: 0 z: .5 } }
           qps { name: "boxwall" pos { x: 10 } } }
defaults { qps { name: "sphere" pos { z: 1.5 } vel { z: 5.0 } }
           qps { name: "sphere_stationary" pos { x: 0 y: 0 z: .5 } }
           qps { name: "boxwall" pos { x: 10 } } }
"""


def _bounce(dev, elasticity, default, steps, dt=None, freeze_ball=False):
  import brax_amd
  from brax_amd import config as cfgmod
  cfg = cfgmod.parse(ELASTIC)
  cfg.elasticity = elasticity
  if dt is not None:
    cfg.dt = dt
  if freeze_ball:
    cfg.bodies[1].frozen.all = True
  s = brax_amd.System(cfg, device=dev)
  qp0 = s.default_qp(default)
  qp = qp0
  for _ in range(steps):
    qp, _ = s.step(qp, torch.zeros(0, device=dev))
  return qp0, qp


@pytest.mark.parametrize('elasticity', [0., .5, 1.])
def test_ball_bounce(dev, elasticity):
  """ElasticityTest (`physics_test.py:863-876`): a capsule hits a frozen box
  wall (capsule-box contacts) and comes back with e^2 of its speed."""
  qp0, qp = _bounce(dev, elasticity, 0, 100)
  places(float(qp0.vel[0][0]) * -1 * elasticity ** 2, qp.vel[0][0], 2)


@pytest.mark.parametrize('elasticity', [0., 1.])
def test_ball_bounce_vertical(dev, elasticity):
  """ElasticityTest (`:878-894`): a ball bounces off another ball."""
  qp0, qp = _bounce(dev, elasticity, 1, 400, dt=2 * 5 / 9.8 / 100.)
  assert abs(float(qp0.vel[0][2]) * elasticity ** 2 - float(qp.vel[0][2])) <= .02


@pytest.mark.parametrize('elasticity', [0., 1.])
def test_ball_bounce_vertical_frozen(dev, elasticity):
  """ElasticityTest (`:896-914`): a ball bounces off a frozen ball."""
  qp0, qp = _bounce(dev, elasticity, 1, 100, dt=2 * 5 / 9.8 / 100., freeze_ball=True)
  assert abs(float(qp0.vel[0][2]) * elasticity ** 2 - float(qp.vel[0][2])) <= .04
