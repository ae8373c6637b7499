"""Normalisation layers (reference: python/paddle/nn/layer/norm.py)."""
import torch

from .layers import Layer
from .. import functional as F
from .. import initializer as I
from ...core.tensor import _wrap


class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-05, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self._normalized_shape = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
        self._epsilon = epsilon
        n = 1
        for s in self._normalized_shape:
            n *= s
        self.weight = self.create_parameter([n], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([n], attr=bias_attr, is_bias=True)

    def forward(self, input):  # noqa: A002
        w, b = self.weight, self.bias
        if len(self._normalized_shape) > 1:
            from ...tensor.manipulation import reshape
            w = reshape(w, self._normalized_shape) if w is not None else None
            b = reshape(b, self._normalized_shape) if b is not None else None
        return F.layer_norm(input, self._normalized_shape, w, b, self._epsilon)

    def extra_repr(self):
        return f"normalized_shape={self._normalized_shape}, epsilon={self._epsilon}"


class RMSNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-05, weight_attr=None, name=None):
        super().__init__()
        self._normalized_shape = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
        self._epsilon = epsilon
        self.weight = self.create_parameter(self._normalized_shape, attr=weight_attr, default_initializer=I.Constant(1.0))

    def forward(self, x):
        return F.rms_norm(x, self._normalized_shape, self.weight, self._epsilon)


class _BatchNormBase(Layer):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None, data_format='NCHW',
                 use_global_stats=None, name=None):
        super().__init__()
        self._num_features, self._momentum, self._epsilon = num_features, momentum, epsilon
        self._data_format, self._use_global_stats = data_format, use_global_stats
        if weight_attr is False:
            self.weight = None
        else:
            self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        if bias_attr is False:
            self.bias = None
        else:
            self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        from ...tensor.creation import zeros, ones
        self.register_buffer('_mean', zeros([num_features], 'float32'))
        self.register_buffer('_variance', ones([num_features], 'float32'))

    def forward(self, input):  # noqa: A002
        return F.batch_norm(input, self._mean, self._variance, self.weight, self.bias, self.training, self._momentum,
                            self._epsilon, self._data_format, self._use_global_stats)

    def extra_repr(self):
        return f"num_features={self._num_features}, momentum={self._momentum}, epsilon={self._epsilon}"


class BatchNorm1D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None, data_format='NCL',
                 use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr,
                         'NC' if data_format in ('NC', 'NCL') else 'NLC', use_global_stats)


class BatchNorm2D(_BatchNormBase):
    pass


class BatchNorm3D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format='NCDHW', use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format, use_global_stats)


class BatchNorm(_BatchNormBase):
    """Legacy paddle.nn.BatchNorm(num_channels, act=None, ...)."""

    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None,
                 bias_attr=None, dtype='float32', data_layout='NCHW', in_place=False, moving_mean_name=None,
                 moving_variance_name=None, do_model_average_for_mean_and_var=True, use_global_stats=False,
                 trainable_statistics=False):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout, use_global_stats or None)
        self._act = act

    def forward(self, input):  # noqa: A002
        y = super().forward(input)
        return getattr(F, self._act)(y) if self._act else y


class SyncBatchNorm(_BatchNormBase):
    """Batch norm whose statistics are all-reduced across the data-parallel group.

    Reference: python/paddle/nn/layer/norm.py SyncBatchNorm (phi sync_batch_norm kernel).
    Here: per-channel (sum, sumsq, count) are all-reduced in ONE fused RCCL call.
    """

    def forward(self, input):  # noqa: A002
        import torch.distributed as dist
        if not self.training or not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
            return super().forward(input)
        return _wrap(_SyncBNFn.apply(input._t, self.weight._t, self.bias._t, self._mean._t, self._variance._t,
                                     self._momentum, self._epsilon, self._data_format))

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        out = layer
        if isinstance(layer, _BatchNormBase) and not isinstance(layer, SyncBatchNorm):
            out = SyncBatchNorm(layer._num_features, layer._momentum, layer._epsilon, data_format=layer._data_format)
            if layer.weight is not None:
                out.weight = layer.weight
                out.bias = layer.bias
            out._mean, out._variance = layer._mean, layer._variance
        for name, sub in layer.named_children():
            out.add_sublayer(name, cls.convert_sync_batchnorm(sub))
        return out


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, rm, rv, momentum, eps, df):
        import torch.distributed as dist
        cl = df[-1] == 'C'
        xc = x.movedim(-1, 1) if cl else x
        dims = [0] + list(range(2, xc.dim()))
        xf = xc.float()
        cnt = torch.tensor([xf.numel() / xf.shape[1]], device=x.device)
        stats = torch.cat([xf.sum(dims), (xf * xf).sum(dims), cnt])
        dist.all_reduce(stats)
        C = xc.shape[1]
        n = stats[-1]
        mean = stats[:C] / n
        var = stats[C:2 * C] / n - mean * mean
        with torch.no_grad():
            rm.mul_(momentum).add_((1 - momentum) * mean)
            rv.mul_(momentum).add_((1 - momentum) * var * n / (n - 1))
        shape = [1, C] + [1] * (xc.dim() - 2)
        inv = torch.rsqrt(var + eps)
        xhat = (xf - mean.view(shape)) * inv.view(shape)
        y = xhat * w.view(shape) + b.view(shape)
        ctx.save_for_backward(xhat, w, inv, n)
        ctx.cl, ctx.dims, ctx.shape = cl, dims, shape
        y = y.to(x.dtype)
        return y.movedim(1, -1) if cl else y

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        xhat, w, inv, n = ctx.saved_tensors
        dyc = (dy.movedim(-1, 1) if ctx.cl else dy).float()
        C = xhat.shape[1]
        red = torch.cat([dyc.sum(ctx.dims), (dyc * xhat).sum(ctx.dims)])
        db_local, dw_local = red[:C].clone(), red[C:].clone()
        dist.all_reduce(red)
        sdy, sdyx = red[:C], red[C:]
        sh = ctx.shape
        dx = (w.view(sh) * inv.view(sh) / n) * (n * dyc - sdy.view(sh) - xhat * sdyx.view(sh))
        dx = dx.to(dy.dtype)
        if ctx.cl:
            dx = dx.movedim(1, -1)
        return dx, dw_local, db_local, None, None, None, None, None


class InstanceNorm1D(Layer):
    _df = 'NCL'

    def __init__(self, num_features, epsilon=1e-05, momentum=0.9, weight_attr=None, bias_attr=None, data_format=None,
                 name=None):
        super().__init__()
        self._eps, self._momentum = epsilon, momentum
        self._data_format = data_format or self._df
        if weight_attr is False:
            self.scale, self.bias = None, None
        else:
            self.scale = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
            self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)

    def forward(self, input):  # noqa: A002
        return F.instance_norm(input, weight=self.scale, bias=self.bias, eps=self._eps, momentum=self._momentum,
                               data_format=self._data_format)


class InstanceNorm2D(InstanceNorm1D):
    _df = 'NCHW'


class InstanceNorm3D(InstanceNorm1D):
    _df = 'NCDHW'


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-05, weight_attr=None, bias_attr=None, data_format='NCHW',
                 name=None):
        super().__init__()
        self._g, self._eps, self._df = num_groups, epsilon, data_format
        self.weight = None if weight_attr is False else self.create_parameter(
            [num_channels], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_channels], attr=bias_attr, is_bias=True)

    def forward(self, input):  # noqa: A002
        return F.group_norm(input, self._g, self._eps, self.weight, self.bias, self._df)


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=0.0001, beta=0.75, k=1.0, data_format='NCHW', name=None):
        super().__init__()
        self._a = (size, alpha, beta, k, data_format)

    def forward(self, x):
        return F.local_response_norm(x, *self._a)


class SpectralNorm(Layer):
    def __init__(self, weight_shape, axis=0, power_iters=1, epsilon=1e-12, dtype='float32'):
        super().__init__()
        self._axis, self._iters, self._eps = axis, power_iters, epsilon
        h = weight_shape[axis]
        w = 1
        for i, s in enumerate(weight_shape):
            if i != axis:
                w *= s
        self.weight_u = self.create_parameter([h], default_initializer=I.Normal(0., 1.))
        self.weight_v = self.create_parameter([w], default_initializer=I.Normal(0., 1.))
        self.weight_u.stop_gradient = True
        self.weight_v.stop_gradient = True

    def forward(self, weight):
        w = weight._t
        wm = w.movedim(self._axis, 0).reshape(w.shape[self._axis], -1)
        u, v = self.weight_u._t, self.weight_v._t
        with torch.no_grad():
            for _ in range(self._iters):
                v.copy_(torch.nn.functional.normalize(wm.t() @ u, dim=0, eps=self._eps))
                u.copy_(torch.nn.functional.normalize(wm @ v, dim=0, eps=self._eps))
        sigma = u @ wm @ v
        return _wrap(w / sigma)
