from . import utils  # noqa: F401


class VectorEnv:
  pass
