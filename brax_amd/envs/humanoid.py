"""Humanoid (upstream `brax/envs/humanoid.py:196-342`) on MI355X.

obs (240) = qpos [torso z, rot, 17 angles] + qvel [vel, ang, 17 joint vels]
+ cinert (11x9) + cvel (11x3) + cang (11x3) + qfrc_actuator (30), where
qfrc uses an UNMASKED take of the padded act_index (-1 reads action[0],
`humanoid.py:318-320`) and cinert adds the INVERSE inertia diagonal.
"""
import numpy as np

from brax_amd import abi
from brax_amd.envs import configs
from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv


class Humanoid(PhysicsEnv):
  """Trains a humanoid to run in the +x direction."""

  kind = 2  # BX_ENV_HUMANOID
  metric_keys = ('distance_from_origin', 'forward_reward', 'reward_alive', 'reward_linvel',
                 'reward_quadctrl', 'x_position', 'x_velocity', 'y_position', 'y_velocity')

  def __init__(self, forward_reward_weight=1.25, ctrl_cost_weight=0.1, healthy_reward=5.0,
               terminate_when_unhealthy=True, healthy_z_range=(0.8, 2.1),
               reset_noise_scale=1e-2, exclude_current_positions_from_observation=True,
               legacy_spring=False, **kwargs):
    # `humanoid.py:209`: legacy_spring selects _SYSTEM_CONFIG_SPRING (three
    # joint groups, no sphericalisation: qfrc is 17 wide there)
    super().__init__(robots.HUMANOID_SPRING_CONFIG if legacy_spring else configs.HUMANOID_CONFIG,
                     **kwargs)
    self.reset_noise_scale = reset_noise_scale
    self.coef = np.array([forward_reward_weight, ctrl_cost_weight, 0, healthy_reward,
                          healthy_z_range[0], healthy_z_range[1],
                          1.0 if terminate_when_unhealthy else 0.0, 0], np.float32)
    # torso x, y lead the obs when positions are included (humanoid.py:289-292)
    self.obs_flags = 0 if exclude_current_positions_from_observation else abi.OBS_XY
    self._set_sizes()
