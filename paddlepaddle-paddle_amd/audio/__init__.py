"""paddle.audio (reference: python/paddle/audio/__init__.py)."""
from . import functional, features, backends  # noqa: F401
from .backends import load, info, save  # noqa: F401


from . import datasets  # noqa: F401,E402


__all__ = ["functional", "features", "datasets", "backends", "load", "info", "save"]
