"""Common layers (reference: python/paddle/nn/layer/common.py, activation.py, distance.py)."""
import numpy as np
import torch

from .layers import Layer
from .. import functional as F
from .. import initializer as I
from ...core.tensor import Tensor, _wrap, _unwrap
from ...framework.param_attr import ParamAttr


class Identity(Layer):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, input):  # noqa: A002
        return input


class Linear(Layer):
    """y = x W + b with W of shape [in_features, out_features]."""

    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self._dtype = self._helper_dtype()
        self.in_features, self.out_features = in_features, out_features
        self.weight = self.create_parameter([in_features, out_features], attr=weight_attr)
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True)
        self.name = name

    def _helper_dtype(self):
        from ...core import dtype as _dt
        return _dt.get_default_dtype()

    def forward(self, input):  # noqa: A002
        return F.linear(input, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, dtype={self._dtype}"


class Bilinear(Layer):
    def __init__(self, in1_features, in2_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([out_features, in1_features, in2_features], attr=weight_attr)
        self.bias = self.create_parameter([1, out_features], attr=bias_attr, is_bias=True)

    def forward(self, x1, x2):
        return F.bilinear(x1, x2, self.weight, self.bias)


class Embedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, max_norm=None, norm_type=2.0, sparse=False,
                 weight_attr=None, name=None):
        super().__init__()
        self._num_embeddings, self._embedding_dim = num_embeddings, embedding_dim
        self._padding_idx = (padding_idx + num_embeddings if padding_idx is not None and padding_idx < 0
                             else padding_idx)
        self._max_norm, self._norm_type, self._sparse = max_norm, norm_type, sparse
        self.weight = self.create_parameter([num_embeddings, embedding_dim], attr=weight_attr)
        if self._padding_idx is not None:
            with torch.no_grad():
                self.weight._t[self._padding_idx] = 0

    def forward(self, x):
        return F.embedding(x, self.weight, self._padding_idx, self._max_norm, self._norm_type, self._sparse)

    def extra_repr(self):
        return f"{self._num_embeddings}, {self._embedding_dim}"


class Dropout(Layer):
    def __init__(self, p=0.5, axis=None, mode='upscale_in_train', name=None):
        super().__init__()
        self.p, self.axis, self.mode = p, axis, mode

    def forward(self, input):  # noqa: A002
        return F.dropout(input, self.p, self.axis, self.training, self.mode)

    def extra_repr(self):
        return f"p={self.p}, axis={self.axis}, mode={self.mode}"


class Dropout2D(Layer):
    def __init__(self, p=0.5, data_format='NCHW', name=None):
        super().__init__()
        self.p, self.data_format = p, data_format

    def forward(self, input):  # noqa: A002
        return F.dropout2d(input, self.p, self.training, self.data_format)


class Dropout3D(Layer):
    def __init__(self, p=0.5, data_format='NCDHW', name=None):
        super().__init__()
        self.p, self.data_format = p, data_format

    def forward(self, input):  # noqa: A002
        return F.dropout3d(input, self.p, self.training, self.data_format)


class AlphaDropout(Layer):
    def __init__(self, p=0.5, name=None):
        super().__init__()
        self.p = p

    def forward(self, input):  # noqa: A002
        return F.alpha_dropout(input, self.p, self.training)


class FeatureAlphaDropout(AlphaDropout):
    def forward(self, input):  # noqa: A002
        return F.feature_alpha_dropout(input, self.p, self.training)


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self.start_axis, self.stop_axis = start_axis, stop_axis

    def forward(self, input):  # noqa: A002
        from ...tensor.manipulation import flatten
        return flatten(input, self.start_axis, self.stop_axis)


class Unflatten(Layer):
    def __init__(self, axis, shape, name=None):
        super().__init__()
        self.axis, self.shape = axis, shape

    def forward(self, input):  # noqa: A002
        from ...tensor.manipulation import unflatten
        return unflatten(input, self.axis, self.shape)


class _PadNd(Layer):
    _nd = 2
    _df = 'NCHW'

    def __init__(self, padding, mode='constant', value=0.0, data_format=None, name=None):
        super().__init__()
        self.padding = [padding] * (2 * self._nd) if isinstance(padding, int) else list(padding)
        self.mode, self.value = mode, value
        self.data_format = data_format or self._df

    def forward(self, x):
        return F.pad(x, self.padding, self.mode, self.value, self.data_format)


class Pad1D(_PadNd):
    _nd, _df = 1, 'NCL'


class Pad2D(_PadNd):
    _nd, _df = 2, 'NCHW'


class Pad3D(_PadNd):
    _nd, _df = 3, 'NCDHW'


class ZeroPad1D(Pad1D):
    def __init__(self, padding, data_format='NCL', name=None):
        super().__init__(padding, 'constant', 0.0, data_format)


class ZeroPad2D(Pad2D):
    def __init__(self, padding, data_format='NCHW', name=None):
        super().__init__(padding, 'constant', 0.0, data_format)


class ZeroPad3D(Pad3D):
    def __init__(self, padding, data_format='NCDHW', name=None):
        super().__init__(padding, 'constant', 0.0, data_format)


class Upsample(Layer):
    def __init__(self, size=None, scale_factor=None, mode='nearest', align_corners=False, align_mode=0,
                 data_format=None, name=None):
        super().__init__()
        self.size, self.scale_factor, self.mode = size, scale_factor, mode
        self.align_corners, self.data_format = align_corners, data_format

    def forward(self, x):
        return F.interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners,
                             data_format=self.data_format)


class UpsamplingNearest2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format='NCHW', name=None):
        super().__init__(size, scale_factor, 'nearest', data_format=data_format)


class UpsamplingBilinear2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format='NCHW', name=None):
        super().__init__(size, scale_factor, 'bilinear', True, data_format=data_format)


class CosineSimilarity(Layer):
    def __init__(self, axis=1, eps=1e-8):
        super().__init__()
        self.axis, self.eps = axis, eps

    def forward(self, x1, x2):
        return F.cosine_similarity(x1, x2, self.axis, self.eps)


class PairwiseDistance(Layer):
    def __init__(self, p=2.0, epsilon=1e-6, keepdim=False, name=None):
        super().__init__()
        self.p, self.epsilon, self.keepdim = p, epsilon, keepdim

    def forward(self, x, y):
        return F.pairwise_distance(x, y, self.p, self.epsilon, self.keepdim)


class Unfold(Layer):
    def __init__(self, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.k, self.d, self.p, self.s = kernel_sizes, dilations, paddings, strides

    def forward(self, x):
        return F.unfold(x, self.k, self.s, self.p, self.d)


class Fold(Layer):
    def __init__(self, output_sizes, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.o, self.k, self.d, self.p, self.s = output_sizes, kernel_sizes, dilations, paddings, strides

    def forward(self, x):
        return F.fold(x, self.o, self.k, self.s, self.p, self.d)


class PixelShuffle(Layer):
    def __init__(self, upscale_factor, data_format='NCHW', name=None):
        super().__init__()
        self.f, self.df = upscale_factor, data_format

    def forward(self, x):
        return F.pixel_shuffle(x, self.f, self.df)


class PixelUnshuffle(Layer):
    def __init__(self, downscale_factor, data_format='NCHW', name=None):
        super().__init__()
        self.f, self.df = downscale_factor, data_format

    def forward(self, x):
        return F.pixel_unshuffle(x, self.f, self.df)


class ChannelShuffle(Layer):
    def __init__(self, groups, data_format='NCHW', name=None):
        super().__init__()
        self.g, self.df = groups, data_format

    def forward(self, x):
        return F.channel_shuffle(x, self.g, self.df)


# ----------------------------------------------------------------------------- activations
def _act(name, fn, argnames=(), defaults=()):
    def __init__(self, *args, **kwargs):
        Layer.__init__(self)
        vals = list(defaults)
        for i, a in enumerate(args[:len(argnames)]):
            vals[i] = a
        for k, v in kwargs.items():
            if k in argnames:
                vals[argnames.index(k)] = v
        self._args = vals

    def forward(self, x):
        return fn(x, *self._args)

    def extra_repr(self):
        return ', '.join(f"{k}={v}" for k, v in zip(argnames, self._args))
    return type(name, (Layer,), {'__init__': __init__, 'forward': forward, 'extra_repr': extra_repr})


ReLU = _act('ReLU', F.relu)
ReLU6 = _act('ReLU6', F.relu6)
Sigmoid = _act('Sigmoid', F.sigmoid)
Tanh = _act('Tanh', F.tanh)
Silu = _act('Silu', F.silu)
Swish = _act('Swish', F.swish)
Mish = _act('Mish', F.mish)
Hardswish = _act('Hardswish', F.hardswish)
Tanhshrink = _act('Tanhshrink', F.tanhshrink)
Softsign = _act('Softsign', F.softsign)
LogSigmoid = _act('LogSigmoid', F.log_sigmoid)
GELU = _act('GELU', F.gelu, ('approximate',), (False,))
ELU = _act('ELU', F.elu, ('alpha',), (1.0,))
CELU = _act('CELU', F.celu, ('alpha',), (1.0,))
SELU = _act('SELU', F.selu, ('scale', 'alpha'), (1.0507009873554804934193349852946, 1.6732632423543772848170429916717))
LeakyReLU = _act('LeakyReLU', F.leaky_relu, ('negative_slope',), (0.01,))
Hardsigmoid = _act('Hardsigmoid', F.hardsigmoid, ('slope', 'offset'), (0.1666667, 0.5))
Hardtanh = _act('Hardtanh', F.hardtanh, ('min', 'max'), (-1.0, 1.0))
Hardshrink = _act('Hardshrink', F.hardshrink, ('threshold',), (0.5,))
Softshrink = _act('Softshrink', F.softshrink, ('threshold',), (0.5,))
Softplus = _act('Softplus', F.softplus, ('beta', 'threshold'), (1, 20))
ThresholdedReLU = _act('ThresholdedReLU', F.thresholded_relu, ('threshold', 'value'), (1.0, 0.0))
Softmax = _act('Softmax', F.softmax, ('axis',), (-1,))
LogSoftmax = _act('LogSoftmax', F.log_softmax, ('axis',), (-1,))
Maxout = _act('Maxout', F.maxout, ('groups', 'axis'), (2, 1))
GLU = _act('GLU', F.glu, ('axis',), (-1,))
RReLU = type('RReLU', (Layer,), {
    '__init__': lambda self, lower=1. / 8., upper=1. / 3., name=None: (Layer.__init__(self), setattr(self, '_lu', (lower, upper)))[0],
    'forward': lambda self, x: F.rrelu(x, self._lu[0], self._lu[1], self.training)})


class Softmax2D(Layer):
    def forward(self, x):
        return F.softmax(x, axis=-3)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format='NCHW', name=None):
        super().__init__()
        self._df = data_format
        self.weight = self.create_parameter([num_parameters], attr=weight_attr, default_initializer=I.Constant(init))

    def forward(self, x):
        return F.prelu(x, self.weight, self._df)
