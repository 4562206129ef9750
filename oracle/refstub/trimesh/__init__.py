from . import exchange  # noqa: F401
