from . import batching  # noqa: F401
