"""paddle.distributed.passes (reference: python/paddle/distributed/passes/__init__.py):
the pass framework (core.py) and the passes over recorded static programs (program_passes.py)."""
from .core import PassBase, PassContext, PassManager, PassType, new_pass, register_pass  # noqa: F401
from . import program_passes  # noqa: F401  (registers the passes)

__all__ = ['new_pass', 'PassManager', 'PassContext']
