"""brax_amd — MI355X-native PBD rigid-body env stepper, drop-in for the
`brax.System.step` / `brax.envs.Env.step/reset` hot path of Prasaya/brax."""

__version__ = '0.1.0'

from brax_amd import config as _config
from brax_amd.base import Info, P, Q, QP
from brax_amd.config import Config
from brax_amd.system import System


def random_prngkey(seed: int):
  """A jax-style (2,) uint32 key for `Env.reset`."""
  import numpy as np  # pylint: disable=import-outside-toplevel
  return np.array([0, seed & 0xFFFFFFFF], dtype=np.uint32)
