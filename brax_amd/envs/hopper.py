"""Hopper and Walker2d (`brax/envs/hopper.py:120-246`, `walker2d.py:130-253`)
on MI355X: one kernel env program (BX_ENV_HOPPER / BX_ENV_WALKER2D) with
each env's constructor defaults.

obs = [torso z, torso pitch (quat_to_euler(rot)[1]), joint angles(D),
torso vel x, vel z, ang y, joint vels(D)], torso x first when
exclude_current_positions_from_observation is False (hopper.py:231-246);
reward = forward_w * dx/dt + healthy_reward - ctrl_w * |a|^2, healthy when
the torso z and pitch are inside their ranges; done = 1 - healthy when
terminate_when_unhealthy (hopper.py:204-229).
"""
import numpy as np

from brax_amd import abi
from brax_amd.envs import robots
from brax_amd.envs.env import PhysicsEnv

_F32_MAX = float(np.finfo(np.float32).max)


def _finite(x):
  """+-inf range ends as +-FLT_MAX: the comparisons keep their outcome for
  every finite state, and the kernels are built without infinities."""
  return float(np.clip(x, -_F32_MAX, _F32_MAX))


class _PlanarWalker(PhysicsEnv):
  # sorted metric names (hopper.py:193-199)
  metric_keys = ('reward_ctrl', 'reward_forward', 'reward_healthy', 'x_position', 'x_velocity')
  config = spring_config = None

  def __init__(self, forward_reward_weight=1.0, ctrl_cost_weight=1e-3, healthy_reward=1.0,
               terminate_when_unhealthy=True, healthy_z_range=(0.7, float('inf')),
               healthy_angle_range=(-0.2, 0.2), reset_noise_scale=5e-3,
               exclude_current_positions_from_observation=True, legacy_spring=False, **kwargs):
    # legacy_spring selects _SYSTEM_CONFIG_SPRING (hopper.py:169)
    super().__init__(self.spring_config if legacy_spring else self.config, **kwargs)
    self.reset_noise_scale = reset_noise_scale
    self.coef = np.array([forward_reward_weight, ctrl_cost_weight, healthy_reward,
                          _finite(healthy_z_range[0]), _finite(healthy_z_range[1]),
                          _finite(healthy_angle_range[0]), _finite(healthy_angle_range[1]),
                          1.0 if terminate_when_unhealthy else 0.0], np.float32)
    self.obs_flags = 0 if exclude_current_positions_from_observation else abi.OBS_XY
    self._set_sizes()


class Hopper(_PlanarWalker):
  """Trains a hopper to hop forward (`brax/envs/hopper.py`)."""
  kind = 5  # BX_ENV_HOPPER
  config = robots.HOPPER_CONFIG
  spring_config = robots.HOPPER_SPRING_CONFIG


class Walker2d(_PlanarWalker):
  """Trains a 2D walker to walk forward (`brax/envs/walker2d.py`; its own
  healthy ranges, walker2d.py:153-163)."""
  kind = 6  # BX_ENV_WALKER2D
  config = robots.WALKER2D_CONFIG
  spring_config = robots.WALKER2D_SPRING_CONFIG

  def __init__(self, healthy_z_range=(0.7, 2.0), healthy_angle_range=(-1.0, 1.0), **kwargs):
    super().__init__(healthy_z_range=healthy_z_range, healthy_angle_range=healthy_angle_range,
                     **kwargs)
