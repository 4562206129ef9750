"""Shared test helpers: systems by name and the parity gate."""
import numpy as np

from brax_amd import compiler
from brax_amd import config as cfgmod
from brax_amd.envs import configs
from brax_amd.envs import robots
from brax_amd.envs.mountain import ant_mountain_config

ENV_CONFIG = {
    'ant': configs.ANT_CONFIG,
    'humanoid': configs.HUMANOID_CONFIG,
    'halfcheetah': configs.HALFCHEETAH_CONFIG,
}


# the other registered envs' pbd systems (physics goldens, oracle/gen_golden.py)
ROBOTS = ['inverted_pendulum', 'inverted_double_pendulum', 'swimmer', 'hopper', 'walker2d',
          'reacher', 'reacherangle', 'acrobot', 'ur5e']


def config_for(name):
  if name in ROBOTS:
    return cfgmod.parse(getattr(robots, name.upper() + '_CONFIG'))
  if name.startswith('mountain'):
    return ant_mountain_config(int(name[len('mountain'):]))
  return cfgmod.parse(ENV_CONFIG[name])


def compiled(name):
  vc, d, meta = compiler.compile_system(config_for(name))
  rd = compiler.compile_reset(vc, meta['body_index'])
  return vc, d, rd, meta


def normwise(a, b):
  """Per-env normwise error max|a-b| / max(1, max|b|) over trailing axes."""
  a = np.asarray(a, np.float64)
  b = np.asarray(b, np.float64)
  axes = tuple(range(1, a.ndim))
  err = np.abs(a - b).max(axis=axes) if axes else np.abs(a - b)
  scale = np.maximum(1.0, np.abs(b).max(axis=axes) if axes else np.abs(b))
  return err / scale


QP_FIELDS = {'pos': slice(0, 3), 'rot': slice(3, 7), 'vel': slice(7, 10), 'ang': slice(10, 13)}
