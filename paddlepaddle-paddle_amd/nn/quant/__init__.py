"""paddle.nn.quant (reference: python/paddle/nn/quant/__init__.py): weight-only / LLM.int8
quantized linear functionals and the quantization ``Stub`` layer."""
from .quantized_linear import (weight_quantize, weight_dequantize, weight_only_linear, llm_int8_linear,  # noqa: F401
                               apply_per_channel_scale)
from .stub import Stub  # noqa: F401

__all__ = ["Stub", "weight_only_linear", "llm_int8_linear", "weight_quantize", "weight_dequantize"]
