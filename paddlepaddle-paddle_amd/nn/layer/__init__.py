"""paddle.nn.layer (reference: python/paddle/nn/layer/__init__.py)."""
from .layers import Layer  # noqa: F401
from .container import Sequential, LayerList, LayerDict, ParameterList, ParameterDict  # noqa: F401
from .common import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .norm import *  # noqa: F401,F403
from .loss import *  # noqa: F401,F403
from .transformer import *  # noqa: F401,F403
from .rnn import *  # noqa: F401,F403
