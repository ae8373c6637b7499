"""paddle.vision (reference: python/paddle/vision/__init__.py)."""
from . import models  # noqa: F401
from .models import *  # noqa: F401,F403
import importlib as _il


def __getattr__(name):
    if name in ('transforms', 'datasets', 'ops', 'image'):
        m = _il.import_module('.' + name, __name__)
        globals()[name] = m
        return m
    raise AttributeError(name)
