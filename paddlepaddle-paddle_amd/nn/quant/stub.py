"""Quantization placeholder layer (reference: python/paddle/nn/quant/stub.py)."""
from ..layer.layers import Layer


class Stub(Layer):
    """Identity placeholder whose ``observer`` (a quanter factory) observes / fake-quantises the
    input once QAT / PTQ replaces it (``paddle.quantization``)."""

    def __init__(self, observer=None):
        super().__init__()
        self._observer = observer

    def forward(self, input):
        return input
