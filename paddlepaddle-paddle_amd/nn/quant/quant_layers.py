"""Dygraph QAT fake-quant layers (the ImperativeQuantAware layer set).

Reference: python/paddle/nn/quant/quant_layers.py (FakeQuantAbsMax:51,
FakeQuantMovingAverageAbsMax:154, FakeQuantChannelWiseAbsMax:292, MovingAverageAbsMaxScale:406,
QuantizedConv2D:522, QuantizedConv2DTranspose:621, QuantizedLinear:739,
QuantizedColumnParallelLinear:816, QuantizedRowParallelLinear:912, QuantizedMatmul:1012,
MAOutputScaleLayer:1071, FakeQuantMAOutputScaleLayer:1105, _get_fake_quant_type:1140) and the
phi kernels behind them (paddle/phi/kernels/funcs/fake_quantize_functor.cu):

  abs_max:        s = max|x|;                         out = round(x / s * R) * s / R
  moving average: state = r*state + 1, accum = r*accum + max|x|, s = accum / state (training;
                  eval uses the stored s); out = round(clip(x / s, -1, 1) * R) * s / R
  channel-wise:   s_c = max|x| over every axis but quant_axis
  R = 2^(bits-1) - 1.  The gradient is straight-through (identity), as the reference's
  fake_quantize_dequantize grad kernels pass dout through.
"""
import torch

from ...core.tensor import Tensor, _wrap, _unwrap
from ..layer.layers import Layer
from .. import functional as F

__all__ = ['FakeQuantAbsMax', 'FakeQuantMovingAverageAbsMax', 'FakeQuantChannelWiseAbsMax', 'QuantizedConv2D',
           'QuantizedConv2DTranspose', 'QuantizedLinear', 'MovingAverageAbsMaxScale', 'MAOutputScaleLayer',
           'FakeQuantMAOutputScaleLayer', 'QuantStub', 'QuantizedRowParallelLinear', 'QuantizedColumnParallelLinear',
           'QuantizedMatmul']


def _rng(bits):
    return float(2 ** (bits - 1) - 1)


def _qdq(x, scale, bits, clip):
    """quant-dequant with a straight-through gradient; scale broadcasts against x."""
    R = _rng(bits)
    s = torch.clamp(scale.to(torch.float32), min=1e-30)
    xf = x.float()
    q = xf / s
    if clip:
        q = torch.clamp(q, -1.0, 1.0)
    y = (torch.round(q * R) * s / R).to(x.dtype)
    return x + (y - x).detach()


def _buf(layer, name, value, dtype='float32'):
    layer.register_buffer(name, _wrap(torch.full([1], float(value), dtype=getattr(torch, dtype))))
    return getattr(layer, name)


def _all_reduce_max(t, reduce_type):
    if reduce_type == 'max':
        import torch.distributed as dist
        if dist.is_initialized():
            dist.all_reduce(t, op=dist.ReduceOp.MAX)


class FakeQuantAbsMax(Layer):
    def __init__(self, name=None, quant_bits=8, dtype='float32', quant_on_weight=False, reduce_type=None):
        super().__init__()
        self._quant_bits = quant_bits
        self._name = name
        self._reduce_type = reduce_type
        self._quant_on_weight = quant_on_weight
        self._scale = _buf(self, '_scale_buf', 0.001, dtype) if quant_on_weight else None

    def forward(self, input):  # noqa: A002
        x = _unwrap(input)
        s = x.detach().abs().max().float().reshape(1)
        _all_reduce_max(s, self._reduce_type)
        if self._scale is not None:
            with torch.no_grad():
                self._scale._t.copy_(s.to(self._scale._t.dtype))
        return _wrap(_qdq(x, s, self._quant_bits, clip=False))


class FakeQuantMovingAverageAbsMax(Layer):
    def __init__(self, name=None, moving_rate=0.9, quant_bits=8, dtype='float32', reduce_type=None):
        super().__init__()
        self._moving_rate = moving_rate
        self._quant_bits = quant_bits
        self._reduce_type = reduce_type
        self._scale = _buf(self, '_scale_buf', 0.001, dtype)
        self._state = _buf(self, '_state_buf', 1, dtype)
        self._accum = _buf(self, '_accum_buf', 1, dtype)

    def forward(self, input):  # noqa: A002
        x = _unwrap(input)
        if self.training:
            with torch.no_grad():
                cur = x.detach().abs().max().float().reshape(1)
                _all_reduce_max(cur, self._reduce_type)
                st, ac, sc = self._state._t, self._accum._t, self._scale._t
                st.mul_(self._moving_rate).add_(1.0)
                ac.mul_(self._moving_rate).add_(cur.to(ac.dtype))
                sc.copy_(ac / st)
        return _wrap(_qdq(x, self._scale._t, self._quant_bits, clip=True))


class FakeQuantChannelWiseAbsMax(Layer):
    def __init__(self, name=None, channel_num=None, quant_bits=8, quant_axis=0, dtype='float32',
                 quant_on_weight=False, reduce_type=None):
        assert quant_on_weight, "Channel_wise only can be used on weight quantization."
        super().__init__()
        self._quant_bits = quant_bits
        self._quant_axis = quant_axis
        self._channel_num = channel_num
        self._reduce_type = reduce_type
        self.register_buffer('_scale_buf', _wrap(torch.full([channel_num], 0.001, dtype=getattr(torch, dtype))))
        self._scale = self._scale_buf

    def forward(self, input):  # noqa: A002
        x = _unwrap(input)
        ax = self._quant_axis % x.dim()
        dims = [d for d in range(x.dim()) if d != ax]
        s = x.detach().abs().float().amax(dim=dims) if dims else x.detach().abs().float()
        _all_reduce_max(s, self._reduce_type)
        with torch.no_grad():
            self._scale._t.copy_(s.to(self._scale._t.dtype))
        shape = [1] * x.dim()
        shape[ax] = -1
        return _wrap(_qdq(x, s.reshape(shape), self._quant_bits, clip=False))


class MovingAverageAbsMaxScale(Layer):
    """Tracks the moving-average abs-max scale of its input; returns the input unchanged."""

    def __init__(self, name=None, moving_rate=0.9, dtype='float32', reduce_type=None):
        super().__init__()
        self._moving_rate = moving_rate
        self._reduce_type = reduce_type
        self._scale = _buf(self, '_scale_buf', 0.0, dtype)
        self._state = _buf(self, '_state_buf', 0.0, dtype)
        self._accum = _buf(self, '_accum_buf', 0.0, dtype)

    def forward(self, input):  # noqa: A002
        x = _unwrap(input)
        if self.training:
            with torch.no_grad():
                cur = x.detach().abs().max().float().reshape(1)
                _all_reduce_max(cur, self._reduce_type)
                st, ac, sc = self._state._t, self._accum._t, self._scale._t
                st.mul_(self._moving_rate).add_(1.0)
                ac.mul_(self._moving_rate).add_(cur.to(ac.dtype))
                sc.copy_(ac / st)
        return input


def _get_fake_quant_type(quant_type, **kwargs):
    call_args = {"name": kwargs.get("name", None), "quant_bits": kwargs.get("quant_bits", 8),
                 "dtype": kwargs.get("dtype", "float32"), "reduce_type": kwargs.get("reduce_type", None)}
    if quant_type == 'abs_max':
        call_args["quant_on_weight"] = kwargs.get("quant_on_weight", False)
    elif quant_type == 'moving_average_abs_max':
        call_args["moving_rate"] = kwargs.get("moving_rate", 0.9)
    elif quant_type == 'channel_wise_abs_max':
        call_args["quant_on_weight"] = kwargs.get("quant_on_weight", False)
        call_args["channel_num"] = kwargs.get("channel_num", None)
        call_args["quant_axis"] = kwargs.get("quant_axis", 0)
        assert call_args["channel_num"] is not None, \
            "You need to input channel_num when you use channel_wise_abs_max strategy."
    elif quant_type in ('lsq_weight', 'channel_wise_lsq_weight'):
        from .lsq import FakeQuantWeightLSQPlus
        per_channel = quant_type == 'channel_wise_lsq_weight'
        return FakeQuantWeightLSQPlus(quant_bits=call_args['quant_bits'], all_positive=kwargs.get('all_positive', False),
                                      per_channel=per_channel,
                                      channel_num=kwargs.get('channel_num', 1) if per_channel else 1,
                                      quant_linear=kwargs.get('quant_linear', False), dtype=call_args['dtype'])
    elif quant_type == 'lsq_act':
        from .lsq import FakeQuantActLSQPlus
        return FakeQuantActLSQPlus(quant_bits=call_args['quant_bits'], all_positive=kwargs.get('all_positive', False),
                                   symmetric=kwargs.get('symmetric', True), dtype=call_args['dtype'])
    fake_quant_map = {'abs_max': FakeQuantAbsMax, 'moving_average_abs_max': FakeQuantMovingAverageAbsMax,
                      'channel_wise_abs_max': FakeQuantChannelWiseAbsMax}
    return fake_quant_map[quant_type](**call_args)


class _QuantWrapped(Layer):
    """Shared construction: weight / activation fake-quant layers and optional pre-layers."""

    def _setup(self, weight, quant_axis, weight_bits, activation_bits, moving_rate, weight_quantize_type,
               activation_quantize_type, weight_pre_layer, act_pre_layer, weight_quant_layer, act_quant_layer,
               act_name=None):
        if weight_quant_layer is not None:
            self._fake_quant_weight = weight_quant_layer()
        else:
            self._fake_quant_weight = _get_fake_quant_type(
                weight_quantize_type, name=getattr(weight, 'name', None), moving_rate=moving_rate,
                quant_bits=weight_bits, quant_on_weight=True, channel_num=weight.shape[quant_axis],
                quant_axis=quant_axis)
        if act_quant_layer is not None:
            self._fake_quant_input = act_quant_layer()
        else:
            self._fake_quant_input = _get_fake_quant_type(activation_quantize_type, name=act_name,
                                                          moving_rate=moving_rate, quant_bits=activation_bits,
                                                          quant_on_weight=False)
        self._act_preprocess = act_pre_layer() if act_pre_layer is not None else None
        self._weight_preprocess = weight_pre_layer() if weight_pre_layer is not None else None

    def _quant_inputs(self, x):
        if self._act_preprocess is not None:
            x = self._act_preprocess(x)
        w = self.weight
        if self._weight_preprocess is not None:
            w = self._weight_preprocess(w)
        return self._fake_quant_input(x), self._fake_quant_weight(w)


_QARGS = dict(weight_bits=8, activation_bits=8, moving_rate=0.9, weight_quantize_type='abs_max',
              activation_quantize_type='abs_max', weight_pre_layer=None, act_pre_layer=None,
              weight_quant_layer=None, act_quant_layer=None)


def _qargs(kw):
    unknown = set(kw) - set(_QARGS)
    if unknown:
        raise TypeError(f"unexpected arguments {sorted(unknown)}")
    a = dict(_QARGS)
    a.update(kw)
    return a


class QuantizedConv2D(_QuantWrapped):
    def __init__(self, layer, **kw):
        super().__init__()
        a = _qargs(kw)
        for k in ('_groups', '_stride', '_padding', '_dilation', '_data_format', '_padding_mode'):
            setattr(self, k, getattr(layer, k, None))
        self._padding_mode = self._padding_mode or 'zeros'
        self._reversed_padding_repeated_twice = getattr(layer, '_reversed_padding_repeated_twice', None)
        self.weight = layer.weight
        self.bias = layer.bias
        self._conv2d_quant_axis = 0
        self._setup(self.weight, 0, act_name=layer.full_name(), **a)

    def forward(self, input):  # noqa: A002
        qx, qw = self._quant_inputs(input)
        padding = self._padding
        if self._padding_mode != 'zeros':
            qx = F.pad(qx, self._reversed_padding_repeated_twice, mode=self._padding_mode,
                       data_format=self._data_format)
            padding = 0
        return F.conv2d(qx, qw, bias=self.bias, padding=padding, stride=self._stride, dilation=self._dilation,
                        groups=self._groups, data_format=self._data_format)


class QuantizedConv2DTranspose(_QuantWrapped):
    def __init__(self, layer, **kw):
        super().__init__()
        a = _qargs(kw)
        for k in ('_groups', '_stride', '_padding', '_dilation', '_data_format', '_output_padding'):
            setattr(self, k, getattr(layer, k, None))
        self.weight = layer.weight
        self.bias = layer.bias
        self._conv2d_transpose_quant_axis = 1
        self._setup(self.weight, 1, act_name=layer.full_name(), **a)

    def forward(self, input, output_size=None):  # noqa: A002
        qx, qw = self._quant_inputs(input)
        return F.conv2d_transpose(qx, qw, bias=self.bias, padding=self._padding,
                                  output_padding=self._output_padding or 0, stride=self._stride,
                                  dilation=self._dilation, groups=self._groups, output_size=output_size,
                                  data_format=self._data_format)


class QuantizedLinear(_QuantWrapped):
    def __init__(self, layer, **kw):
        super().__init__()
        a = _qargs(kw)
        self.weight = layer.weight
        self.bias = layer.bias
        self.name = getattr(layer, '_name', None)
        self._linear_quant_axis = 1
        self._setup(self.weight, 1, act_name=layer.full_name(), **a)

    def forward(self, input):  # noqa: A002
        qx, qw = self._quant_inputs(input)
        return F.linear(qx, qw, self.bias)


class QuantizedColumnParallelLinear(_QuantWrapped):
    def __init__(self, layer, **kw):
        super().__init__()
        a = _qargs(kw)
        assert a['weight_quant_layer'] is None, "When quantizing ColumnParallelLinear, weight_quant_layer should be None."
        assert a['act_quant_layer'] is None, "When quantizing ColumnParallelLinear, act_quant_layer should be None."
        self.weight = layer.weight
        self.bias = layer.bias
        self._layer = layer
        self.is_mp = layer.is_mp
        self.model_parallel_group = layer.model_parallel_group
        self.gather_output = layer.gather_output
        self._linear_quant_axis = 1
        self._setup(self.weight, 1, act_name=layer.full_name(), **a)

    def forward(self, input):  # noqa: A002
        from ...distributed.fleet.layers.mpu import mp_ops
        x = input
        if self.is_mp:
            x = mp_ops._c_identity(x, group=self.model_parallel_group)
        qx, qw = self._quant_inputs(x)
        out = F.linear(qx, qw, self.bias)
        if self.gather_output and self.is_mp:
            out = mp_ops._c_concat(out, group=self.model_parallel_group)
        return out


class QuantizedRowParallelLinear(_QuantWrapped):
    def __init__(self, layer, **kw):
        super().__init__()
        a = _qargs(kw)
        assert a['weight_quant_layer'] is None, "When quantizing RowParallelLinear, weight_quant_layer cannot defined by yourself."
        assert a['act_quant_layer'] is None, "When quantizing RowParallelLinear, act_quant_layer cannot defined by yourself."
        self.weight = layer.weight
        self.bias = layer.bias
        self.is_mp = layer.is_mp
        self.model_parallel_group = layer.model_parallel_group
        self.input_is_parallel = layer.input_is_parallel
        self._linear_quant_axis = 1
        self._setup(self.weight, 1, act_name=layer.full_name(), **a)

    def forward(self, input):  # noqa: A002
        from ...distributed.fleet.layers.mpu import mp_ops
        x = input
        if self.is_mp and not self.input_is_parallel:
            x = mp_ops._c_split(x, group=self.model_parallel_group)
        qx, qw = self._quant_inputs(x)
        out = F.linear(qx, qw, None)
        if self.is_mp:
            out = mp_ops._mp_allreduce(out, group=self.model_parallel_group)
        if self.bias is not None:
            out = out + self.bias
        return out


class QuantizedMatmul(Layer):
    def __init__(self, layer=None, **kw):
        super().__init__()
        a = _qargs(kw)
        if a['act_quant_layer'] is not None:
            self._fake_quant_x = a['act_quant_layer']()
            self._fake_quant_y = a['act_quant_layer']()
        else:
            mk = lambda: _get_fake_quant_type(a['activation_quantize_type'], moving_rate=a['moving_rate'],  # noqa: E731
                                              quant_bits=a['activation_bits'], quant_on_weight=False)
            self._fake_quant_x, self._fake_quant_y = mk(), mk()
        pre = a['act_pre_layer']
        self._act_preprocess_x = pre() if pre is not None else None
        self._act_preprocess_y = pre() if pre is not None else None

    def forward(self, x, y, transpose_x=False, transpose_y=False, name=None):
        from ...tensor.linalg import matmul
        if self._act_preprocess_x is not None:
            x = self._act_preprocess_x(x)
        if self._act_preprocess_y is not None:
            y = self._act_preprocess_y(y)
        return matmul(self._fake_quant_x(x), self._fake_quant_y(y), transpose_x, transpose_y)


class MAOutputScaleLayer(Layer):
    def __init__(self, layer=None, moving_rate=0.9, name=None, dtype='float32', reduce_type=None):
        super().__init__()
        self._layer = layer
        if name is None and layer is not None:
            name = layer.full_name()
        self._ma_output_scale = MovingAverageAbsMaxScale(name, moving_rate, dtype, reduce_type)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple, dict)):
            return out
        return self._ma_output_scale(out)


class FakeQuantMAOutputScaleLayer(Layer):
    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, name=None, reduce_type=None,
                 *args, **kwargs):
        super().__init__()
        self._layer = layer
        self._fake_quant_output = _get_fake_quant_type(
            'moving_average_abs_max', name=layer.full_name() if name is None else name, moving_rate=moving_rate,
            quant_bits=activation_bits, quant_on_weight=False, reduce_type=reduce_type)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple)) and len(out) > 1:
            return out
        return self._fake_quant_output(out)


class QuantStub(Layer):
    """Fake-quantises its input (placed where a float model enters a quantised region)."""

    def __init__(self, activation_quantize_type='moving_average_abs_max', moving_rate=0.9, activation_bits=8,
                 act_quant_layer=None, **kw):
        super().__init__()
        if act_quant_layer is not None:
            self._fake_quant = act_quant_layer()
        else:
            self._fake_quant = _get_fake_quant_type(activation_quantize_type, moving_rate=moving_rate,
                                                    quant_bits=activation_bits, quant_on_weight=False)

    def forward(self, input):  # noqa: A002
        return self._fake_quant(input)


def _is_tensor(x):
    return isinstance(x, Tensor)
