"""Shared test helpers: systems by name and the parity gate."""
import numpy as np

from brax_amd import compiler
from brax_amd import config as cfgmod
from brax_amd.envs import configs
from brax_amd.envs import robots
from brax_amd.envs.mountain import ant_mountain_config

ENV_CONFIG = {
    'humanoidstandup': robots.HUMANOID_STANDUP_CONFIG,
    'ant': configs.ANT_CONFIG,
    'humanoid': configs.HUMANOID_CONFIG,
    'halfcheetah': configs.HALFCHEETAH_CONFIG,
}


# the other registered envs' pbd systems (physics goldens, oracle/gen_golden.py)
ROBOTS = ['inverted_pendulum', 'inverted_double_pendulum', 'swimmer', 'hopper', 'walker2d',
          'reacher', 'reacherangle', 'acrobot', 'ur5e', 'pusher', 'grasp', 'fetch']


# the CapsuleTest scene (reference `brax/tests/physics_test.py:292-328`) as
# test input data; variants 'ground', 'capsule', 'cull' as in its three tests
CAPSULE_TEST_CONFIG = """
dt: 20.0 substeps: 10000 friction: 0.6 gravity { z: -9.8 }
bodies { name: "Capsule1" mass: 1 colliders { capsule { radius: 0.25 length: 1.0 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Capsule2" mass: 1 colliders { rotation { y: 90 } capsule { radius: 0.25 length: 1.0 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Capsule3" mass: 1 colliders { rotation { y: 45 } capsule { radius: 0.25 length: 1.0 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Capsule4" mass: 1 colliders { rotation { x: 45 } capsule { radius: 0.25 length: 1.0 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "Ground" frozen { all: true } colliders { plane {} } }
defaults { qps { name: "Capsule1" pos { z: 1 } } qps { name: "Capsule2" pos { x: 1 z: 1 } } qps { name: "Capsule3" pos { x: 3 z: 1 } } qps { name: "Capsule4" pos { x: 5 z: 1 } } }
defaults { qps { name: "Capsule1" pos { z: 1 } } qps { name: "Capsule2" pos { z: 2 } } qps { name: "Capsule3" pos { x: 3 z: 1 } } qps { name: "Capsule4" pos { x: 5 z: 1 } } }
"""
CAPSULES = ['capsule_ground', 'capsule_capsule', 'capsule_cull']
# short-horizon twins of the long physics-test scenes (dt 0.05, 10 substeps,
# from a state falling into contact; oracle/gen_golden.py _short_scenes):
# the golden trajectory gates run on these, the long scenes stay KATs
SHORT_SCENES = ['capsule_ground_s', 'capsule_capsule_s', 'capsule_cull_s', 'box_ground_s',
                'box_slide_s']
# NearNeighbors with more cutoff than allowed cells: top_k also returns
# masked cells (oracle/scenes.py TWIN_CULL_CONFIG; golden generated under
# jax.lax.top_k's tie order)
NN_MASKED = ['twin_cull']
# legacy_spring systems (`_SYSTEM_CONFIG_SPRING`, system.py:342-390): envs with
# the kernel env layer, and physics rollouts of the other registered envs
SPRING_ENVS = ['ant_spring', 'humanoid_spring', 'halfcheetah_spring', 'humanoidstandup_spring']
SPRING_ROBOTS = [m + '_spring' for m in (
    'inverted_pendulum', 'inverted_double_pendulum', 'swimmer', 'hopper', 'walker2d', 'reacher',
    'reacherangle', 'acrobot', 'ur5e', 'grasp', 'fetch')]
_SPRING_MOD = {'halfcheetah': 'HALF_CHEETAH', 'humanoidstandup': 'HUMANOID_STANDUP'}


# exclude_current_positions_from_observation=False rollouts (traj_<env>_xy)
XY_ENVS = ['ant_xy', 'humanoid_xy', 'halfcheetah_xy']


# kernel env kinds whose reference rollouts are the envtraj_* goldens (the
# env-layer rollouts of oracle/gen_golden.py) rather than traj_*
ENVTRAJ_KERNEL = ['hopper', 'walker2d', 'inverted_pendulum', 'inverted_double_pendulum', 'acrobot',
                  'reacher', 'reacherangle', 'swimmer', 'pusher', 'ur5e', 'fetch', 'grasp']
# bodies a kernel env's reset places after default_qp (reacher.py:177-179,
# pusher.py:196-201): name -> body names


def reset_bodies(name):
  return {'reacher': ['target'], 'reacherangle': ['target'], 'ur5e': ['Target'],
          'fetch': ['Target'], 'pusher': ['goal', 'object', 'table']}.get(name, [])


def env_coef(name):
  """bx_env_params.coef of a kernel env with its constructor defaults, built
  on the CPU (None: the oracle's built-in defaults apply)."""
  from brax_amd.envs import tasks
  if name in ('reacher', 'reacherangle'):
    cfg = config_for(name)
    return tasks.reacher_coef(cfg, compiled(name)[3]['body_index'], angle=name == 'reacherangle')
  if name == 'swimmer':
    return tasks.swimmer_coef()
  if name == 'pusher':
    return tasks.pusher_coef(compiled(name)[3]['body_index'])
  if name == 'grasp':
    return tasks.grasp_coef(compiled(name)[3]['body_index'])
  if name in ('ur5e', 'fetch'):
    cls = tasks.Ur5e if name == 'ur5e' else tasks.Fetch
    return tasks.target_coef(compiled(name)[3]['body_index'], cls.torso, *cls.ring)
  return None


def prep_oracle(o, name):
  """Per-env oracle state: Grasp's action map."""
  if name == 'grasp':
    from brax_amd.envs import tasks
    o.set_act_map(tasks.grasp_act_map(config_for(name)))
  return o


def golden_reset_qp(name, o, T):
  """The oracle's default_qp of the golden reset angles, with the bodies the
  env's reset places copied from the golden's reset state."""
  qp0 = o.default_qp(T['reset_qpos'], T['reset_qvel'])
  idx = [compiled(name)[3]['body_index'][b] for b in reset_bodies(name)]
  for b in idx:
    qp0[:, b, 0:3] = T['qp'][0][:, b, 0:3]
  return qp0


def env_golden(name):
  """Golden file of a kernel env's reference rollout."""
  return ('envtraj_' if name in ENVTRAJ_KERNEL else 'traj_') + name


def env_kind(name):
  """Env-layer kind of a golden name ('ant_spring', 'ant_xy' -> 'ant')."""
  for suf in ('_spring', '_xy'):
    if name.endswith(suf):
      return name[:-len(suf)]
  return name


def obs_flags(name):
  """BX_OBS_* of a golden name (abi.OBS_XY for the *_xy rollouts)."""
  return 1 if name.endswith('_xy') else 0


# point-plane scenes: BoxTest (box corners) and an inline-mesh MeshTest
# (mesh vertices), oracle/scenes.py
POINTS = ['box_ground', 'box_slide', 'mesh_ground', 'mesh_tilt']
# the extended contact functions' scenes (oracle/scenes.py): box corners on a
# height map, spheres on a clipped plane, capsules against box / mesh triangles
XCOL = ['heightmap', 'clipped', 'box_capsule', 'mesh_capsule', 'box_box', 'box_capsule_hull']


def config_for(name):
  if name in SHORT_SCENES:
    base = name[:-2]
    cfg = config_for('box_ground' if base.startswith('box') else base)
    cfg.dt, cfg.substeps = 0.05, 10
    return cfg
  if name.endswith('_xy'):
    name = name[:-len('_xy')]
  if name.endswith('_spring'):
    base = name[:-len('_spring')]
    return cfgmod.parse(getattr(robots, _SPRING_MOD.get(base, base.upper()) + '_SPRING_CONFIG'))
  if name in CAPSULES:
    cfg = cfgmod.parse(CAPSULE_TEST_CONFIG)
    if name != 'capsule_ground':
      cfg.dt = 2.0
      cfg.substeps = 400
    if name == 'capsule_cull':
      cfg.collider_cutoff = 1
    return cfg
  if name in XCOL:
    from oracle import scenes
    return cfgmod.parse({'heightmap': lambda: scenes.heightmap_config(0.05, 10),
                         'clipped': lambda: scenes.clipped_plane_config(0.05, 10),
                         'box_capsule': lambda: scenes.BOX_CAPSULE_NO_HULL_CONFIG,
                         'mesh_capsule': scenes.mesh_capsule_config,
                         'box_box': lambda: scenes.box_box_config(0.05, 20),
                         'box_capsule_hull': lambda: scenes.BOX_CAPSULE_TEST_CONFIG}[name]())
  if name in POINTS:
    from oracle import scenes
    return cfgmod.parse(scenes.BOX_TEST_CONFIG if name.startswith('box')
                        else scenes.mesh_test_config())
  if name == 'twin_cull':
    from oracle import scenes
    return cfgmod.parse(scenes.TWIN_CULL_CONFIG)
  if name in ('mountain1nn', 'mountain2nn', 'mountain4nn'):
    n = int(name[len('mountain')])
    cfg = ant_mountain_config(n)
    cfg.collider_cutoff = 9 * n
    return cfg
  if name in ROBOTS:
    return cfgmod.parse(getattr(robots, name.upper() + '_CONFIG'))
  if name.startswith('mountain'):
    return ant_mountain_config(int(name[len('mountain'):]))
  return cfgmod.parse(ENV_CONFIG[name])


def compiled(name):
  vc, d, meta = compiler.compile_system(config_for(name))
  rd = compiler.compile_reset(vc, meta['body_index'])
  return vc, d, rd, meta


def set_variant(sys_, variant):
  """Put a System on one large-scene kernel: 'multi' (the MULTI kernel at its
  own width: 128 threads per env where the scene fits, else 256), 'multi256'
  (the MULTI kernel at 256 threads per env), 'itemloop' / 'items' (the item
  loops at 256 threads per env). Returns bx_system_set_variant's status."""
  from brax_amd import _native
  lib = _native.lib()
  if variant == 'multi':
    rc = lib.bx_system_set_variant(sys_._h, 128, 3)
    return rc if rc == 0 else lib.bx_system_set_variant(sys_._h, 256, 3)
  if variant == 'multi256':
    return lib.bx_system_set_variant(sys_._h, 256, 3)
  return lib.bx_system_set_variant(sys_._h, 256, 0)


def normwise(a, b):
  """Per-env normwise error max|a-b| / max(1, max|b|) over trailing axes."""
  a = np.asarray(a, np.float64)
  b = np.asarray(b, np.float64)
  axes = tuple(range(1, a.ndim))
  err = np.abs(a - b).max(axis=axes) if axes else np.abs(a - b)
  scale = np.maximum(1.0, np.abs(b).max(axis=axes) if axes else np.abs(b))
  return err / scale


QP_FIELDS = {'pos': slice(0, 3), 'rot': slice(3, 7), 'vel': slice(7, 10), 'ang': slice(10, 13)}
