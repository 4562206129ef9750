"""Ant (`brax/envs/ant.py:173-286`): reward, observation and reset on MI355X.

obs = [torso z, torso rot(4), joint angles(8), torso vel(3), torso ang(3),
joint vels(8), clip(contact.vel)(10x3), clip(contact.ang)(10x3)] = 87 with
use_contact_forces (the registered 'ant'), else 27 (`ant.py:257-282`); torso
x, y lead it when exclude_current_positions_from_observation is False.
"""
import numpy as np

from brax_amd import abi
from brax_amd.envs import configs
from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv


class Ant(PhysicsEnv):
  """Trains an ant to run in the +x direction."""

  kind = 1  # BX_ENV_ANT
  # sorted metric names (`ant.py:207-219`)
  metric_keys = ('distance_from_origin', 'forward_reward', 'reward_contact', 'reward_ctrl',
                 'reward_forward', 'reward_survive', 'x_position', 'x_velocity',
                 'y_position', 'y_velocity')

  def __init__(self, ctrl_cost_weight=0.5, use_contact_forces=False, contact_cost_weight=5e-4,
               healthy_reward=1.0, terminate_when_unhealthy=True, healthy_z_range=(0.2, 1.0),
               reset_noise_scale=0.1, exclude_current_positions_from_observation=True,
               legacy_spring=False, **kwargs):
    # `ant.py:183-184`: legacy_spring selects _SYSTEM_CONFIG_SPRING
    super().__init__(robots.ANT_SPRING_CONFIG if legacy_spring else configs.ANT_CONFIG, **kwargs)
    self.reset_noise_scale = reset_noise_scale
    self._use_contact_forces = use_contact_forces
    self.coef = np.array([1.0, ctrl_cost_weight, contact_cost_weight, healthy_reward,
                          healthy_z_range[0], healthy_z_range[1],
                          1.0 if terminate_when_unhealthy else 0.0,
                          1.0 if use_contact_forces else 0.0], np.float32)
    # exclude_current_positions_from_observation=False: torso x, y lead the
    # obs (ant.py:262-265)
    self.obs_flags = 0 if exclude_current_positions_from_observation else abi.OBS_XY
    self._set_sizes()
