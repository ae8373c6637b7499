"""paddle.nn.initializer (reference: python/paddle/nn/initializer/*.py).

Initializers fill a Parameter's storage in place under no_grad. fan_in/fan_out follow
paddle's convention for Linear weights stored ``[in_features, out_features]`` and conv
weights ``[out_c, in_c/groups, kh, kw]``.
"""
import math

import numpy as np
import torch

from ..core.tensor import Tensor, _unwrap

_global_weight_init = None
_global_bias_init = None


def _fans(shape):
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[2:]))
    return shape[1] * rf, shape[0] * rf


def calculate_gain(nonlinearity, param=None):
    g = {'sigmoid': 1.0, 'linear': 1.0, 'conv1d': 1.0, 'conv2d': 1.0, 'conv3d': 1.0, 'conv1d_transpose': 1.0,
         'conv2d_transpose': 1.0, 'conv3d_transpose': 1.0, 'tanh': 5.0 / 3, 'relu': math.sqrt(2.0),
         'selu': 3.0 / 4}
    if nonlinearity == 'leaky_relu':
        p = 0.01 if param is None else param
        return math.sqrt(2.0 / (1 + p ** 2))
    return g[nonlinearity]


class Initializer:
    def __call__(self, param, block=None):
        t = _unwrap(param)
        with torch.no_grad():
            self._init(t)
        return param

    def _init(self, t):
        raise NotImplementedError

    forward = __call__


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def _init(self, t):
        t.fill_(self.value)


ConstantInitializer = Constant


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        if t.dtype in (torch.bfloat16, torch.float16):
            t.copy_(torch.empty_like(t, dtype=torch.float32).normal_(self.mean, self.std))
        else:
            t.normal_(self.mean, self.std)


NormalInitializer = Normal


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, a=-2.0, b=2.0, name=None):
        self.mean, self.std, self.a, self.b = mean, std, a, b

    def _init(self, t):
        tmp = torch.empty_like(t, dtype=torch.float32)
        torch.nn.init.trunc_normal_(tmp, self.mean, self.std, self.mean + self.a * self.std, self.mean + self.b * self.std)
        t.copy_(tmp)


TruncatedNormalInitializer = TruncatedNormal


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, name=None):
        self.low, self.high = low, high

    def _init(self, t):
        tmp = torch.empty_like(t, dtype=torch.float32) if t.dtype != torch.float64 else t
        tmp.uniform_(self.low, self.high)
        if tmp is not t:
            t.copy_(tmp)


UniformInitializer = Uniform


class XavierNormal(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        std = self.gain * math.sqrt(2.0 / float(fi + fo))
        Normal(0.0, std)._init(t)


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        lim = self.gain * math.sqrt(6.0 / float(fi + fo))
        Uniform(-lim, lim)._init(t)


XavierInitializer = XavierUniform


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity='relu', mode='fan_in'):
        self.fan_in, self.slope, self.nl, self.mode = fan_in, negative_slope, nonlinearity, mode

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        f = self.fan_in or (fi if self.mode == 'fan_in' else fo)
        std = calculate_gain(self.nl, self.slope) / math.sqrt(f)
        Normal(0.0, std)._init(t)


MSRAInitializer = KaimingNormal


class KaimingUniform(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity='relu', mode='fan_in'):
        self.fan_in, self.slope, self.nl, self.mode = fan_in, negative_slope, nonlinearity, mode

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        f = self.fan_in or (fi if self.mode == 'fan_in' else fo)
        lim = calculate_gain(self.nl, self.slope) * math.sqrt(3.0 / f)
        Uniform(-lim, lim)._init(t)


class Assign(Initializer):
    def __init__(self, value, name=None):
        self.value = value

    def _init(self, t):
        v = _unwrap(self.value) if isinstance(self.value, Tensor) else torch.as_tensor(np.asarray(self.value))
        t.copy_(v.reshape(t.shape).to(t.dtype))


NumpyArrayInitializer = Assign


class Orthogonal(Initializer):
    def __init__(self, gain=1.0, name=None):
        self.gain = gain

    def _init(self, t):
        tmp = torch.empty(t.shape[0], int(np.prod(t.shape[1:])), dtype=torch.float32)
        torch.nn.init.orthogonal_(tmp, self.gain)
        t.copy_(tmp.reshape(t.shape))


class Dirac(Initializer):
    def __init__(self, groups=1, name=None):
        self.groups = groups

    def _init(self, t):
        tmp = torch.empty(t.shape, dtype=torch.float32)
        torch.nn.init.dirac_(tmp, self.groups)
        t.copy_(tmp)


class Bilinear(Initializer):
    def _init(self, t):
        shape = list(t.shape)
        size = shape[3]
        f = math.ceil(size / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = np.zeros(shape, dtype=np.float32)
        for i in range(int(np.prod(shape))):
            x = i % size
            y = (i / size) % shape[2]
            w.flat[i] = (1 - abs(x / f - c)) * (1 - abs(y / f - c))
        t.copy_(torch.from_numpy(w))


def set_global_initializer(weight_init, bias_init=None):
    global _global_weight_init, _global_bias_init
    _global_weight_init, _global_bias_init = weight_init, bias_init


def _global_init(is_bias):
    return _global_bias_init if is_bias else _global_weight_init


def _register_lazy_init():
    """``paddle.nn.initializer.lazy_init`` (reference: nn/initializer/lazy_init.py: LazyGuard)."""
    import sys
    import types
    from ..framework import LazyGuard
    m = types.ModuleType(__name__ + '.lazy_init')
    m.LazyGuard = LazyGuard
    m.__all__ = ['LazyGuard']
    sys.modules[m.__name__] = m
    return m


lazy_init = _register_lazy_init()
