"""paddle.nn (reference: python/paddle/nn/__init__.py)."""
from .layer import *  # noqa: F401,F403
from .layer.layers import Layer  # noqa: F401
from . import functional, initializer, utils, quant  # noqa: F401
from .clip import ClipGradByValue, ClipGradByNorm, ClipGradByGlobalNorm  # noqa: F401
from ..core.tensor import Parameter  # noqa: F401
from .decode import BeamSearchDecoder, dynamic_decode  # noqa: F401
