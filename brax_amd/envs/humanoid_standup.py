"""HumanoidStandup (`brax/envs/humanoid_standup.py:210-297`) on MI355X.

The Humanoid observation program (240 dims, `humanoid_standup.py:249-290`)
on its own system (lying start, 22 contact rows); reward = torso z / dt + 1
- 0.01 sum(a^2); done is left as it came in. One fused kernel launch
(env kind BX_ENV_HUMANOID_STANDUP).
"""
import numpy as np

from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv


class HumanoidStandup(PhysicsEnv):
  """Trains a humanoid to stand up."""

  kind = 4  # BX_ENV_HUMANOID_STANDUP
  metric_keys = ('reward_linup', 'reward_quadctrl')

  def __init__(self, legacy_spring=False, **kwargs):
    # `humanoid_standup.py:213`: legacy_spring selects _SYSTEM_CONFIG_SPRING
    super().__init__(robots.HUMANOID_STANDUP_SPRING_CONFIG if legacy_spring
                     else robots.HUMANOID_STANDUP_CONFIG, **kwargs)
    self.reset_noise_scale = 0.01
    self.coef = np.array([0, 0.01, 0, 0, 0, 0, 0, 0], np.float32)
    self._set_sizes()
