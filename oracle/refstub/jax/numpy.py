"""Sentinel `jax.numpy`: only `ndarray` is needed, as an isinstance target."""


class ndarray:  # pylint: disable=invalid-name
  pass
