"""Conv / pooling layers (reference: python/paddle/nn/layer/{conv,pooling}.py)."""
import numpy as np

from .layers import Layer
from .. import functional as F
from .. import initializer as I


def _nt(v, n):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


class _ConvNd(Layer):
    _nd = 2
    _transpose = False
    _fn = None

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode='zeros', weight_attr=None, bias_attr=None, data_format=None, output_padding=0):
        super().__init__()
        nd = self._nd
        self._in, self._out = in_channels, out_channels
        self._k = _nt(kernel_size, nd)
        self._stride, self._padding, self._dilation, self._groups = stride, padding, dilation, groups
        self._padding_mode = padding_mode
        self._output_padding = output_padding
        self._data_format = data_format or {1: 'NCL', 2: 'NCHW', 3: 'NCDHW'}[nd]
        if self._transpose:
            shape = [in_channels, out_channels // groups] + list(self._k)
        else:
            shape = [out_channels, in_channels // groups] + list(self._k)
        fan_in = int(np.prod(shape[1:]))
        std = (2.0 / fan_in) ** 0.5
        self.weight = self.create_parameter(shape, attr=weight_attr, default_initializer=I.Normal(0.0, std))
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True)

    def _maybe_pad(self, x):
        if self._padding_mode == 'zeros':
            return x, self._padding
        p = _nt(self._padding, self._nd)
        pads = []
        for v in reversed(p):
            pads += [v, v]
        mode = {'reflect': 'reflect', 'replicate': 'replicate', 'circular': 'circular'}[self._padding_mode]
        return F.pad(x, pads, mode, data_format=self._data_format), 0

    def forward(self, x, output_size=None):
        if self._transpose:
            fn = {1: F.conv1d_transpose, 2: F.conv2d_transpose, 3: F.conv3d_transpose}[self._nd]
            if self._nd == 2:
                return fn(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                          self._dilation, self._groups, output_size, self._data_format)
            return fn(x, self.weight, self.bias, self._stride, self._padding, self._output_padding, self._groups,
                      self._dilation, output_size, self._data_format)
        fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[self._nd]
        x, p = self._maybe_pad(x)
        return fn(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups, self._data_format)

    def extra_repr(self):
        return (f"{self._in}, {self._out}, kernel_size={list(self._k)}, stride={self._stride}, "
                f"padding={self._padding}, data_format={self._data_format}")


def _conv_cls(name, nd, transpose):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, *args, **kwargs):
        if transpose:
            names = ['output_padding', 'groups', 'dilation', 'weight_attr', 'bias_attr', 'data_format'] if nd != 2 else \
                ['output_padding', 'dilation', 'groups', 'weight_attr', 'bias_attr', 'data_format']
        else:
            names = ['dilation', 'groups', 'padding_mode', 'weight_attr', 'bias_attr', 'data_format']
        kw = dict(zip(names, args))
        kw.update(kwargs)
        kw.pop('name', None)
        _ConvNd.__init__(self, in_channels, out_channels, kernel_size, stride, padding, **kw)
    return type(name, (_ConvNd,), {'_nd': nd, '_transpose': transpose, '__init__': __init__})


Conv1D = _conv_cls('Conv1D', 1, False)
Conv2D = _conv_cls('Conv2D', 2, False)
Conv3D = _conv_cls('Conv3D', 3, False)
Conv1DTranspose = _conv_cls('Conv1DTranspose', 1, True)
Conv2DTranspose = _conv_cls('Conv2DTranspose', 2, True)
Conv3DTranspose = _conv_cls('Conv3DTranspose', 3, True)


class _Pool(Layer):
    def __init__(self, fn, **kw):
        super().__init__()
        self._fn, self._kw = fn, kw

    def forward(self, x):
        return self._fn(x, **self._kw)

    def extra_repr(self):
        return ', '.join(f"{k}={v}" for k, v in self._kw.items())


def _pool_cls(name, fn, argnames):
    def __init__(self, *args, **kwargs):
        kw = dict(zip(argnames, args))
        kw.update({k: v for k, v in kwargs.items() if k != 'name'})
        _Pool.__init__(self, fn, **kw)
    return type(name, (_Pool,), {'__init__': __init__})


MaxPool1D = _pool_cls('MaxPool1D', F.max_pool1d, ['kernel_size', 'stride', 'padding', 'return_mask', 'ceil_mode'])
MaxPool2D = _pool_cls('MaxPool2D', F.max_pool2d, ['kernel_size', 'stride', 'padding', 'return_mask', 'ceil_mode',
                                                  'data_format'])
MaxPool3D = _pool_cls('MaxPool3D', F.max_pool3d, ['kernel_size', 'stride', 'padding', 'return_mask', 'ceil_mode',
                                                  'data_format'])
AvgPool1D = _pool_cls('AvgPool1D', F.avg_pool1d, ['kernel_size', 'stride', 'padding', 'exclusive', 'ceil_mode'])
AvgPool2D = _pool_cls('AvgPool2D', F.avg_pool2d, ['kernel_size', 'stride', 'padding', 'ceil_mode', 'exclusive',
                                                  'divisor_override', 'data_format'])
AvgPool3D = _pool_cls('AvgPool3D', F.avg_pool3d, ['kernel_size', 'stride', 'padding', 'ceil_mode', 'exclusive',
                                                  'divisor_override', 'data_format'])
AdaptiveAvgPool1D = _pool_cls('AdaptiveAvgPool1D', F.adaptive_avg_pool1d, ['output_size'])
AdaptiveAvgPool2D = _pool_cls('AdaptiveAvgPool2D', F.adaptive_avg_pool2d, ['output_size', 'data_format'])
AdaptiveAvgPool3D = _pool_cls('AdaptiveAvgPool3D', F.adaptive_avg_pool3d, ['output_size', 'data_format'])
AdaptiveMaxPool1D = _pool_cls('AdaptiveMaxPool1D', F.adaptive_max_pool1d, ['output_size', 'return_mask'])
AdaptiveMaxPool2D = _pool_cls('AdaptiveMaxPool2D', F.adaptive_max_pool2d, ['output_size', 'return_mask'])
AdaptiveMaxPool3D = _pool_cls('AdaptiveMaxPool3D', F.adaptive_max_pool3d, ['output_size', 'return_mask'])
LPPool1D = _pool_cls('LPPool1D', F.lp_pool1d, ['norm_type', 'kernel_size', 'stride', 'ceil_mode', 'data_format'])
LPPool2D = _pool_cls('LPPool2D', F.lp_pool2d, ['norm_type', 'kernel_size', 'stride', 'ceil_mode', 'data_format'])
FractionalMaxPool2D = _pool_cls('FractionalMaxPool2D', F.fractional_max_pool2d, ['output_size', 'kernel_size',
                                                                                  'random_u', 'return_mask'])
FractionalMaxPool3D = _pool_cls('FractionalMaxPool3D', F.fractional_max_pool3d, ['output_size', 'kernel_size',
                                                                                  'random_u', 'return_mask'])


class _Unpool(Layer):
    _fn = None

    def __init__(self, kernel_size, stride=None, padding=0, data_format=None, output_size=None, name=None):
        super().__init__()
        self._a = (kernel_size, stride, padding)
        self._os = output_size

    def forward(self, x, indices):
        return type(self)._fn(x, indices, *self._a, output_size=self._os)


class MaxUnPool1D(_Unpool):
    _fn = staticmethod(F.max_unpool1d)


class MaxUnPool2D(_Unpool):
    _fn = staticmethod(F.max_unpool2d)


class MaxUnPool3D(_Unpool):
    _fn = staticmethod(F.max_unpool3d)
