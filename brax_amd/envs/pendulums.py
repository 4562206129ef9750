"""InvertedPendulum, InvertedDoublePendulum and Acrobot on MI355X: kernel env
programs BX_ENV_INVERTED_PENDULUM / _DOUBLE_PENDULUM / ACROBOT.

* InvertedPendulum (`inverted_pendulum.py:133-164`): obs = [cart x, joint
  angle, cart vel x, joint vel]; reward 1; done when |angle| > .2. Its one
  action drives a 3-wide Thruster whose indices clip to action[0].
* InvertedDoublePendulum (`inverted_double_pendulum.py:140-184`): obs =
  [cart x, sin(angles), cos(angles), cart vel x, joint vels]; reward =
  10 - (.01 x^2 + (y - 2)^2) - (1e-3 v1^2 + 5e-3 v2^2) at the pole tip
  (body 2's (0, 0, .3) in the world); done when the tip's z <= 1.
* Acrobot (`acrobot.py:56-95`): obs = [joint angles, joint vels]; reward =
  10 - |angles|^2 - 1e-3 |vels|^2; never done.

Reset: default angles + U[-.01, .01) joint noise, U[-.01, .01) velocities.
"""
from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv


class _OneActionEnv(PhysicsEnv):
  config = spring_config = None
  reset_noise_scale = 0.01

  def __init__(self, legacy_spring=False, **kwargs):
    super().__init__(self.spring_config if legacy_spring else self.config, **kwargs)
    self._set_sizes()

  @property
  def action_size(self):
    return 1


class InvertedPendulum(_OneActionEnv):
  kind = 7  # BX_ENV_INVERTED_PENDULUM
  config = robots.INVERTED_PENDULUM_CONFIG
  spring_config = robots.INVERTED_PENDULUM_SPRING_CONFIG


class InvertedDoublePendulum(_OneActionEnv):
  kind = 8  # BX_ENV_INVERTED_DOUBLE_PENDULUM
  config = robots.INVERTED_DOUBLE_PENDULUM_CONFIG
  spring_config = robots.INVERTED_DOUBLE_PENDULUM_SPRING_CONFIG


class Acrobot(_OneActionEnv):
  kind = 9  # BX_ENV_ACROBOT
  config = robots.ACROBOT_CONFIG
  spring_config = robots.ACROBOT_SPRING_CONFIG
  # sorted metric names (acrobot.py:70-75)
  metric_keys = ('alive_bonus', 'dist_penalty', 'r_tot', 'vel_penalty')
