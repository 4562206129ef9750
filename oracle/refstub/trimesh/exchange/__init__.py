from . import load  # noqa: F401
