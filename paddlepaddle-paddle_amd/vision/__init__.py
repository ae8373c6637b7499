"""paddle.vision (reference: python/paddle/vision/__init__.py)."""
from . import models  # noqa: F401
from .models import *  # noqa: F401,F403
import importlib as _il


def set_image_backend(backend):
    from .image import set_image_backend as f
    return f(backend)


def get_image_backend():
    from .image import get_image_backend as f
    return f()


def image_load(path, backend=None):
    from .image import image_load as f
    return f(path, backend)


def __getattr__(name):
    if name in ('transforms', 'datasets', 'ops', 'image'):
        m = _il.import_module('.' + name, __name__)
        globals()[name] = m
        return m
    raise AttributeError(name)
