from . import specs  # noqa: F401
import enum


class Environment:
  pass


class StepType(enum.IntEnum):
  FIRST = 0
  MID = 1
  LAST = 2


class TimeStep(tuple):
  pass
