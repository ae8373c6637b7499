"""paddle.incubate (reference: python/paddle/incubate/__init__.py)."""
from . import nn  # noqa: F401
