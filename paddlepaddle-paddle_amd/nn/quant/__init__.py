"""paddle.nn.quant (reference: python/paddle/nn/quant/__init__.py): weight-only / LLM.int8
quantized linear functionals and the quantization ``Stub`` layer."""
from .quantized_linear import (weight_quantize, weight_dequantize, weight_only_linear, llm_int8_linear,  # noqa: F401
                               apply_per_channel_scale)
from .stub import Stub  # noqa: F401
from . import quant_layers, lsq, functional_layers  # noqa: F401
from .functional_layers import (add, subtract, multiply, divide, reshape, transpose, concat,  # noqa: F401
                                flatten, matmul, FloatFunctionalLayer)
from .quant_layers import (FakeQuantAbsMax, FakeQuantMovingAverageAbsMax, FakeQuantChannelWiseAbsMax,  # noqa: F401
                           QuantizedConv2D, QuantizedConv2DTranspose, QuantizedLinear, MovingAverageAbsMaxScale,
                           MAOutputScaleLayer, FakeQuantMAOutputScaleLayer, QuantStub, QuantizedRowParallelLinear,
                           QuantizedColumnParallelLinear, QuantizedMatmul)
from .lsq import FakeQuantActLSQPlus, FakeQuantWeightLSQPlus  # noqa: F401

__all__ = ["Stub", "weight_only_linear", "llm_int8_linear", "weight_quantize", "weight_dequantize"]
