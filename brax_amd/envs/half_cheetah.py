"""HalfCheetah (`brax/envs/half_cheetah.py:147-218`) on MI355X.

obs = [torso z, rot.w, rot.y, joint angles(6), vel.x, vel.z, ang.y,
joint vels(6)] = 18; reward = forward_w * dx/dt - ctrl_w * |a|^2; never done.
"""
import numpy as np

from brax_amd import abi
from brax_amd.envs import configs
from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv


class Halfcheetah(PhysicsEnv):
  """Trains a halfcheetah to run in the +x direction."""

  kind = 3  # BX_ENV_HALFCHEETAH
  metric_keys = ('reward_ctrl', 'reward_run', 'x_position', 'x_velocity')

  def __init__(self, forward_reward_weight=1.0, ctrl_cost_weight=0.1, reset_noise_scale=0.1,
               legacy_spring=False, exclude_current_positions_from_observation=True, **kwargs):
    # `half_cheetah.py:154`: legacy_spring selects _SYSTEM_CONFIG_SPRING
    super().__init__(robots.HALF_CHEETAH_SPRING_CONFIG if legacy_spring
                     else configs.HALFCHEETAH_CONFIG, **kwargs)
    self.reset_noise_scale = reset_noise_scale
    self.coef = np.array([forward_reward_weight, ctrl_cost_weight, 0, 0, 0, 0, 0, 0], np.float32)
    # torso x leads z when positions are included (half_cheetah.py:206-209)
    self.obs_flags = 0 if exclude_current_positions_from_observation else abi.OBS_XY
    self._set_sizes()
