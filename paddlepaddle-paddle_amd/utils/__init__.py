"""paddle.utils (reference: python/paddle/utils/__init__.py)."""
from . import unique_name  # noqa: F401
from . import cpp_extension  # noqa: F401
from .dlpack_utils import to_dlpack, from_dlpack  # noqa: F401
from . import dlpack_utils as dlpack  # noqa: F401
from .install_check import run_check  # noqa: F401
from .deprecated import deprecated  # noqa: F401
from . import download  # noqa: F401


def try_import(module_name, err_msg=None):
    import importlib
    try:
        return importlib.import_module(module_name)
    except ImportError as e:
        raise ImportError(err_msg or f"{module_name} is required but not installed") from e


def require_version(min_version, max_version=None):
    return True


def flops(net, input_size, custom_ops=None, print_detail=False):
    from ..hapi.dynamic_flops import flops as _f
    return _f(net, input_size, custom_ops, print_detail)


def disable_signal_handler():
    """The reference installs C++ signal handlers; this framework installs none."""
    return None


def check_shape(shape, op_name='', expected_shape_type=(list, tuple), expected_element_type=(int,),
                expected_tensor_dtype=('int32', 'int64')):
    if not isinstance(shape, expected_shape_type) and not hasattr(shape, 'shape'):
        raise TypeError(f"{op_name}: shape must be list/tuple/Tensor, got {type(shape)}")
    if isinstance(shape, (list, tuple)):
        for s in shape:
            if not isinstance(s, expected_element_type) and not hasattr(s, 'shape'):
                raise TypeError(f"{op_name}: shape elements must be int, got {type(s)}")
