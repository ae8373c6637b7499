"""paddle.tensor namespace (reference: python/paddle/tensor/__init__.py)."""
from .creation import *  # noqa: F401,F403
from .math import *  # noqa: F401,F403
from .manipulation import *  # noqa: F401,F403
from .linalg import *  # noqa: F401,F403
from .logic import *  # noqa: F401,F403
from . import creation, math, manipulation, linalg, logic  # noqa: F401
from ..core.tensor import Tensor, to_tensor, is_tensor  # noqa: F401


def _public(mod):
    return {k: v for k, v in vars(mod).items() if not k.startswith('_') and callable(v)
            and getattr(v, '__module__', '').startswith(mod.__name__)}


def all_functions():
    d = {}
    for m in (creation, math, manipulation, linalg, logic):
        d.update(_public(m))
    return d
