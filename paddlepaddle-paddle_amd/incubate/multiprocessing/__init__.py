"""paddle.incubate.multiprocessing — the standard ``multiprocessing`` module with paddle Tensors
picklable through shared memory (reference: python/paddle/incubate/multiprocessing/__init__.py)."""
from multiprocessing import *  # noqa: F401,F403

from .reductions import init_reductions

__all__ = []

init_reductions()
