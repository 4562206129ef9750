"""Sentinel `jax.core`: the reference asks only for the trace level."""


class _Level:
  level = 0


def cur_sublevel():
  return _Level()
