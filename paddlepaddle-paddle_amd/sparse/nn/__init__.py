"""paddle.sparse.nn layers (reference: python/paddle/sparse/nn/layer/*.py)."""
import math

import torch

from ...nn.layer.layers import Layer
from ...nn import initializer as I
from ...core.tensor import _wrap, _unwrap
from . import functional  # noqa: F401
from . import functional as SF


class ReLU(Layer):
    def forward(self, x):
        return SF.relu(x)


class ReLU6(Layer):
    def forward(self, x):
        return SF.relu6(x)


class LeakyReLU(Layer):
    def __init__(self, negative_slope=0.01, name=None):
        super().__init__()
        self._slope = negative_slope

    def forward(self, x):
        return SF.leaky_relu(x, self._slope)


class Softmax(Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__()
        self._axis = axis

    def forward(self, x):
        return SF.softmax(x, self._axis)


class BatchNorm(Layer):
    """BatchNorm over the channel (last) dim of the stored values of a COO tensor."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format='NDHWC', use_global_stats=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        self.register_buffer('_mean', _wrap(torch.zeros(num_features)))
        self.register_buffer('_variance', _wrap(torch.ones(num_features)))
        self._momentum, self._epsilon = momentum, epsilon
        self._use_global_stats = use_global_stats

    def _norm(self, v):
        rm, rv = self._mean._t, self._variance._t
        if self.training and not self._use_global_stats:
            mean, var = v.mean(0), v.var(0, unbiased=False)
            self._sync(mean, var, v.shape[0])
            with torch.no_grad():
                rm.mul_(self._momentum).add_((1 - self._momentum) * mean.detach())
                rv.mul_(self._momentum).add_((1 - self._momentum) * var.detach())
        else:
            mean, var = rm, rv
        return (v - mean) / torch.sqrt(var + self._epsilon) * self.weight._t + self.bias._t

    def _sync(self, mean, var, n):
        return None

    def forward(self, x):
        t = _unwrap(x).coalesce()
        return _wrap(torch.sparse_coo_tensor(t.indices(), self._norm(t.values()), t.shape).coalesce())


class SyncBatchNorm(BatchNorm):
    """Statistics all-reduced across the data-parallel group (one fused [sum, sumsq, n] reduce)."""

    def _norm(self, v):
        import torch.distributed as dist
        if not (self.training and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return super()._norm(v)
        stats = torch.cat([v.sum(0), (v * v).sum(0), torch.tensor([float(v.shape[0])], device=v.device)])
        dist.all_reduce(stats)
        C = v.shape[1]
        n = stats[-1]
        mean = stats[:C] / n
        var = stats[C:2 * C] / n - mean * mean
        with torch.no_grad():
            self._mean._t.mul_(self._momentum).add_((1 - self._momentum) * mean)
            self._variance._t.mul_(self._momentum).add_((1 - self._momentum) * var)
        return (v - mean) / torch.sqrt(var + self._epsilon) * self.weight._t + self.bias._t

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        for name, sub in list(layer._sub_layers.items()):
            if isinstance(sub, BatchNorm) and not isinstance(sub, SyncBatchNorm):
                new = cls.__new__(cls)
                new.__dict__.update(sub.__dict__)
                layer._sub_layers[name] = new
            else:
                cls.convert_sync_batchnorm(sub)
        return layer


class _Conv(Layer):
    def __init__(self, nd, subm, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode='zeros', key=None, weight_attr=None, bias_attr=None, data_format=None):
        super().__init__()
        ks = (kernel_size,) * nd if isinstance(kernel_size, int) else tuple(kernel_size)
        fan_in = in_channels // groups * int(math.prod(ks))
        self.weight = self.create_parameter(list(ks) + [in_channels // groups, out_channels], attr=weight_attr,
                                            default_initializer=I.Uniform(-1 / math.sqrt(fan_in),
                                                                          1 / math.sqrt(fan_in)))
        self.bias = None if bias_attr is False else self.create_parameter([out_channels], attr=bias_attr,
                                                                          is_bias=True)
        self._nd, self._subm = nd, subm
        self._stride, self._padding, self._dilation, self._groups = stride, padding, dilation, groups

    def forward(self, x):
        return SF._conv(x, self.weight, self.bias, 1 if self._subm else self._stride, self._padding, self._dilation,
                        self._groups, self._subm, self._nd, None)


class Conv2D(_Conv):
    def __init__(self, *a, **k):
        super().__init__(2, False, *a, **k)


class Conv3D(_Conv):
    def __init__(self, *a, **k):
        super().__init__(3, False, *a, **k)


class SubmConv2D(_Conv):
    def __init__(self, *a, **k):
        super().__init__(2, True, *a, **k)


class SubmConv3D(_Conv):
    def __init__(self, *a, **k):
        super().__init__(3, True, *a, **k)


class MaxPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format="NDHWC", name=None):
        super().__init__()
        self._k, self._s, self._p = kernel_size, stride, padding

    def forward(self, x):
        return SF.max_pool3d(x, self._k, self._s, self._p)


__all__ = ['ReLU', 'ReLU6', 'LeakyReLU', 'Softmax', 'BatchNorm', 'SyncBatchNorm', 'Conv2D', 'Conv3D', 'SubmConv2D',
           'SubmConv3D', 'MaxPool3D']
