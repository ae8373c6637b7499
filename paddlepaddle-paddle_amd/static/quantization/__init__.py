"""paddle.static.quantization — post-training quantisation and quantisation-aware training passes
for static Programs (reference: python/paddle/static/quantization/__init__.py).  Frozen int8 GEMMs
run on the int8 MFMA kernel (csrc/gemm8x.hip pa_gemm8_i8)."""
from .passes import (  # noqa: F401
    QuantizationTransformPass, QuantizationTransformPassV2, QuantizationFreezePass, ConvertToInt8Pass,
    AddQuantDequantPass, AddQuantDequantPassV2, AddQuantDequantForInferencePass, OutScaleForTrainingPass,
    OutScaleForInferencePass, QuantWeightPass, ReplaceFakeQuantDequantPass, TransformForMobilePass, find_sites,
)
from .post_training import (  # noqa: F401
    PostTrainingQuantization, PostTrainingQuantizationProgram, WeightQuantization,
)
from .quanter import quant_aware, convert  # noqa: F401


class _OneDNNOnly:
    """The oneDNN (x86 CPU) int8 graph passes of the reference; this runtime's int8 path is the
    MI355X int8 MFMA GEMM of QuantizationFreezePass / PostTrainingQuantization."""

    def __init__(self, *a, **k):
        raise NotImplementedError(f"{type(self).__name__} targets oneDNN on x86 CPUs; freeze with "
                                  "QuantizationFreezePass for the MI355X int8 kernels")


class QuantInt8MkldnnPass(_OneDNNOnly):
    pass


class Quant2Int8MkldnnPass(_OneDNNOnly):
    pass


__all__ = []
