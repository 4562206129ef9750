from . import host_callback  # noqa: F401
