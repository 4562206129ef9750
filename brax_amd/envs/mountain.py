"""Ant Mountain: the multi-agent contact stress scene of the reference's
`notebooks/multiagent.ipynb` (cell 3): `count` Ants cloned from the Ant config,
dropped in a spiral, every collision pair on (630 capsule-capsule pairs at 4)."""
import copy

import numpy as np

from brax_amd import config as cfgmod
from brax_amd.envs import configs


def ant_mountain_config(count: int, cutoff: int = 0):
  config = cfgmod.parse(configs.ANT_CONFIG)
  repeat = count - 1
  for lst in (config.bodies, config.joints, config.actuators):
    for obj in list(lst):
      if obj.name == 'Ground':
        continue
      for i in range(repeat):
        new_obj = lst.add()
        new_obj.CopyFrom(obj)
        for attr in ('name', 'joint', 'parent', 'child'):
          if attr in cfgmod._SCHEMA[new_obj._type]:  # pylint: disable=protected-access
            setattr(new_obj, attr, f'{getattr(new_obj, attr)}_{i}')
  default = config.defaults.add()
  for i in range(repeat):
    qp = default.qps.add(name=f'$ Torso_{i}')
    qp.pos.x = np.sin(i * np.pi / 2)
    qp.pos.y = np.cos(i * np.pi / 2)
    qp.pos.z = (i + 1) * 2
  del config.collide_include[:]
  config.collider_cutoff = cutoff
  return config


def ant_mountain(count: int, cutoff: int = 0, device=None):
  from brax_amd.system import System  # pylint: disable=import-outside-toplevel
  return System(ant_mountain_config(count, cutoff), device=device)
