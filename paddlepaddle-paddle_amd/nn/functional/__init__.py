"""paddle.nn.functional (reference: python/paddle/nn/functional/__init__.py)."""
from .activation import *  # noqa: F401,F403
from .common import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .norm import *  # noqa: F401,F403
from .loss import *  # noqa: F401,F403
from .flash_attention import (flash_attention, flash_attn_qkvpacked, flash_attn_unpadded, masked_attention_bhsd,  # noqa: F401,E501
                              flash_attn_varlen_qkvpacked,
                              scaled_dot_product_attention, flash_attention_with_sparse_mask, sparse_attention,
                              memory_efficient_attention)
from ...tensor.math import sigmoid, tanh  # noqa: F401
from ...tensor.creation import diag_embed  # noqa: F401
from ...tensor.manipulation import unfold as _unfold_t  # noqa: F401
from .common import unfold  # noqa: F401,F811
