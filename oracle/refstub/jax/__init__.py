"""Test-only stand-in for the `jax` package.

It exists solely so that the reference's own numpy backend
(`brax/jumpy.py:16-48`, which dispatches to numpy whenever no jax array is
involved) can be imported in this container to generate golden vectors.
Nothing here is a JAX implementation: `_which_np` always sees plain numpy
arrays, so every reference op runs in numpy float64.
Never imported by the product package.
"""
import functools as _ft

from . import tree_util  # noqa: F401
from . import numpy  # noqa: F401
from . import core  # noqa: F401
from . import interpreters  # noqa: F401


class _Config:
  jax_disable_jit = False


config = _Config()


class custom_jvp:  # pylint: disable=invalid-name
  """Pass-through decorator with a no-op `.defjvp`."""

  def __init__(self, fun):
    self.fun = fun
    _ft.update_wrapper(self, fun)

  def __call__(self, *a, **k):
    return self.fun(*a, **k)

  def defjvp(self, jvp):
    return jvp
