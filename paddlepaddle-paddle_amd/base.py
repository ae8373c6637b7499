"""paddle.base (reference: python/paddle/base/): the legacy "fluid" namespace, mapped onto this
framework's core modules."""
from .framework import in_dynamic_mode, enable_static, disable_static  # noqa: F401
from .static import (Program, program_guard, default_main_program, default_startup_program, Executor,  # noqa: F401
                     global_scope, scope_guard, CompiledProgram, BuildStrategy, ExecutionStrategy)
from .core.place import CPUPlace, CUDAPlace, CUDAPinnedPlace  # noqa: F401
from .framework.param_attr import ParamAttr  # noqa: F401
from . import core as core  # noqa: F401
from .autograd import no_grad  # noqa: F401


class dygraph:  # noqa: N801
    from .autograd import no_grad  # noqa: F401
    from .core.tensor import to_tensor as to_variable  # noqa: F401

    @staticmethod
    def guard(place=None):
        import contextlib
        return contextlib.nullcontext()


def create_lod_tensor(data, recursive_seq_lens, place=None):
    """paddle.base.create_lod_tensor (level-1 LoD on a Tensor; static/sequence.py)."""
    from .static.sequence import create_lod_tensor as _c
    return _c(data, recursive_seq_lens, place)
