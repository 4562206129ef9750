from . import spaces  # noqa: F401
from . import vector  # noqa: F401


class Env:
  pass


class Wrapper(Env):
  def __init__(self, env):
    self.env = env
