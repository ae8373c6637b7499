"""Functional ops as layers, so QAT passes can wrap them (reference:
python/paddle/nn/quant/functional_layers.py)."""
from ..layer.layers import Layer


class FloatFunctionalLayer(Layer):
    def __init__(self):
        super().__init__()


def _mk(fname, doc):
    def forward(self, *args, **kwargs):
        import paddle
        return getattr(paddle, fname)(*args, **kwargs)
    cls = type(fname, (FloatFunctionalLayer,), {'forward': forward, '__doc__': doc})
    return cls


add = _mk('add', "paddle.add as a layer")
subtract = _mk('subtract', "paddle.subtract as a layer")
multiply = _mk('multiply', "paddle.multiply as a layer")
divide = _mk('divide', "paddle.divide as a layer")
reshape = _mk('reshape', "paddle.reshape as a layer")
transpose = _mk('transpose', "paddle.transpose as a layer")
concat = _mk('concat', "paddle.concat as a layer")
flatten = _mk('flatten', "paddle.flatten as a layer")
matmul = _mk('matmul', "paddle.matmul as a layer")
