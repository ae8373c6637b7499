"""paddle.incubate.nn (reference: python/paddle/incubate/nn/__init__.py)."""
from . import functional  # noqa: F401
from .layer import (FusedEcMoe, FusedLinear, FusedDropoutAdd, FusedFeedForward, FusedMultiHeadAttention,  # noqa: F401
                    FusedTransformerEncoderLayer, FusedMultiTransformer, FusedBiasDropoutResidualLayerNorm)
