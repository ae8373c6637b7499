"""paddle.jit (reference: python/paddle/jit/__init__.py)."""
from .api import (to_static, not_to_static, save, load, ignore_module, TranslatedLayer,  # noqa: F401
                  enable_to_static, set_code_level, set_verbosity, StaticFunction)
from ..static.program import InputSpec  # noqa: F401
from . import sot  # noqa: F401

__all__ = ['save', 'load', 'to_static', 'ignore_module', 'TranslatedLayer', 'set_code_level', 'set_verbosity',
           'not_to_static', 'enable_to_static']
