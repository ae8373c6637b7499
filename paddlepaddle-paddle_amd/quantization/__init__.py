"""paddle.quantization (reference: python/paddle/quantization/{config,qat,ptq,quantize,factory,
base_quanter,base_observer}.py, quanters/abs_max.py, observers/abs_max.py).

QAT inserts fake quant-dequant (moving-average abs-max scales, straight-through gradient)
on the weights and inputs of Linear / Conv layers; PTQ inserts abs-max observers, and
``convert`` freezes observed scales into fixed quant-dequant ops.  ``convert(...,
to_fp8=True)`` additionally swaps Linear layers for e4m3 GEMMs (MI355X fp8 MFMA path,
``ops/gemm.py``) using the observed per-tensor scales.
"""
import abc
import copy
import functools

import torch

from ..nn.layer.layers import Layer
from ..nn import Linear, Conv2D, Conv1D, Conv3D
from ..core.tensor import Tensor, _wrap, _unwrap


# ----------------------------------------------------------------- factories
class ClassWithArguments(metaclass=abc.ABCMeta):
    def __init__(self, *args, **kwargs):
        self._args = args
        self._kwargs = kwargs

    @property
    def args(self):
        return self._args

    @property
    def kwargs(self):
        return self._kwargs

    @abc.abstractmethod
    def _get_class(self):
        pass

    def __str__(self):
        return f"{self._get_class().__name__}({', '.join(map(str, self._args))})"


class QuanterFactory(ClassWithArguments):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.partial_class = None

    def _instance(self, layer):
        if self.partial_class is None:
            self.partial_class = functools.partial(self._get_class(), *self.args, **self.kwargs)
        return self.partial_class(layer)


ObserverFactory = QuanterFactory


def quanter(class_name):
    """Decorator: registers ``class_name`` as a factory for the decorated quanter layer."""
    def wrapper(target_class):
        import sys
        factory = type(class_name, (QuanterFactory,), {'_get_class': lambda self: target_class})
        mod = sys.modules[target_class.__module__]
        setattr(mod, class_name, factory)
        return target_class
    return wrapper


class BaseQuanter(Layer, metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def forward(self, input):  # noqa: A002
        pass

    @abc.abstractmethod
    def scales(self):
        pass

    @abc.abstractmethod
    def zero_points(self):
        pass

    @abc.abstractmethod
    def quant_axis(self):
        pass

    @abc.abstractmethod
    def bit_length(self):
        pass


class BaseObserver(BaseQuanter, metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def cal_thresholds(self):
        pass


# ----------------------------------------------------------------- fake quant kernels
class _FakeQuant(torch.autograd.Function):
    """round(clip(x / s, -1, 1) * q) * s / q with a straight-through gradient inside the range."""

    @staticmethod
    def forward(ctx, x, scale, qmax):
        s = scale.clamp(min=1e-9).to(x.dtype)
        y = torch.round(torch.clamp(x / s, -1.0, 1.0) * qmax) * s / qmax
        ctx.save_for_backward((x.abs() <= s).to(x.dtype))
        return y

    @staticmethod
    def backward(ctx, g):
        m, = ctx.saved_tensors
        return g * m, None, None


def fake_quant_dequant(x, scale, bit_length=8):
    return _FakeQuant.apply(x, scale, float(2 ** (bit_length - 1) - 1))


class FakeQuanterWithAbsMaxObserverLayer(BaseQuanter):
    def __init__(self, layer=None, name=None, moving_rate=0.9, bit_length=8, dtype='float32'):
        super().__init__()
        self._moving_rate = moving_rate
        self._bit_length = bit_length
        self.register_buffer('_scale', _wrap(torch.full([1], 0.001)))
        self.register_buffer('_state', _wrap(torch.ones([1])))
        self.register_buffer('_accum', _wrap(torch.ones([1])))

    def forward(self, input):  # noqa: A002
        x = _unwrap(input)
        sc, st, ac = self._scale._t, self._state._t, self._accum._t
        if self.training:
            with torch.no_grad():
                cur = x.detach().abs().max().float().reshape(1).to(sc.device)
                st.mul_(self._moving_rate).add_(1.0)
                ac.mul_(self._moving_rate).add_(cur)
                sc.copy_(ac / st)
        return _wrap(fake_quant_dequant(x, sc.to(x.device), self._bit_length))

    def bit_length(self):
        return self._bit_length

    def quant_axis(self):
        return -1

    def scales(self):
        return self._scale

    def zero_points(self):
        return None


class FakeQuanterWithAbsMaxObserver(QuanterFactory):
    def __init__(self, moving_rate=0.9, bit_length=8, dtype='float32', name=None):
        super().__init__(name=name, moving_rate=moving_rate, bit_length=bit_length, dtype=dtype)

    def _get_class(self):
        return FakeQuanterWithAbsMaxObserverLayer


class AbsmaxObserverLayer(BaseObserver):
    """Records max |x| over calibration batches; passes x through unchanged."""

    def __init__(self, layer=None, quant_bits=8):
        super().__init__()
        self._quant_bits = quant_bits
        self.register_buffer('_max', _wrap(torch.zeros([1])))

    def forward(self, input):  # noqa: A002
        x = _unwrap(input)
        with torch.no_grad():
            m = self._max._t
            m.copy_(torch.maximum(m, x.detach().abs().max().float().reshape(1).to(m.device)))
        return input

    def cal_thresholds(self):
        return self._max

    def bit_length(self):
        return self._quant_bits

    def quant_axis(self):
        return -1

    def scales(self):
        return self._max

    def zero_points(self):
        return None


class AbsmaxObserver(ObserverFactory):
    def __init__(self, quant_bits=8):
        super().__init__(quant_bits=quant_bits)

    def _get_class(self):
        return AbsmaxObserverLayer


class GroupWiseWeightObserverLayer(BaseObserver):
    """Per-group abs-max of a 2-D [in, out] weight: groups of ``group_size`` input rows, one
    scale per (group, output column) — reference quantization/observers/groupwise.py."""

    def __init__(self, layer=None, quant_bits=8, group_size=128):
        super().__init__()
        self._quant_bits = quant_bits
        self.group_size = group_size
        self._max = None
        self._scale = None
        self._zero_point = None

    def forward(self, inputs):
        self._max = self._cal_abs_max(inputs)
        return inputs

    def _cal_abs_max(self, inputs):
        x = _unwrap(inputs)
        assert self.group_size in (64, 128), "group_size only support 64 or 128"
        assert x.dim() == 2, "Currently only support 2D tensor"
        assert x.shape[0] % self.group_size == 0, "group_size must be a factor of input channels"
        g = x.detach().t().reshape(x.shape[1], x.shape[0] // self.group_size, self.group_size)
        m = g.abs().amax(dim=2).float()
        m = torch.where(m == 0, torch.full_like(m, 1e-8), m)
        return _wrap(m.t().contiguous())

    def min_value(self):
        return 0.0

    def max_value(self):
        return self._max

    def bit_length(self):
        return self._quant_bits

    def quant_axis(self):
        return -1

    def cal_thresholds(self):
        if self._scale is None:
            self._scale = self._max
        self._zero_point = _wrap(torch.zeros_like(_unwrap(self._scale)))

    def scales(self):
        if self._scale is None:
            self.cal_thresholds()
        return self._scale

    def zero_points(self):
        if self._zero_point is None:
            self.cal_thresholds()
        return self._zero_point


class GroupWiseWeightObserver(ObserverFactory):
    def __init__(self, quant_bits=8, group_size=128):
        super().__init__(quant_bits=quant_bits, group_size=group_size)

    def _get_class(self):
        return GroupWiseWeightObserverLayer


class LinearQuanterDequanter(Layer):
    """Frozen quant-dequant with a fixed scale (what ``convert`` leaves in the model)."""

    def __init__(self, scale, bit_length=8):
        super().__init__()
        self.register_buffer('scale', _wrap(_unwrap(scale).detach().clone().float()))
        self._bits = bit_length

    def forward(self, x):
        t = _unwrap(x)
        return _wrap(fake_quant_dequant(t, self.scale._t.to(t.device), self._bits))


# ----------------------------------------------------------------- config
class SingleLayerConfig:
    def __init__(self, activation, weight):
        self._activation = activation
        self._weight = weight

    @property
    def activation(self):
        return self._activation

    @property
    def weight(self):
        return self._weight

    def __str__(self):
        return f"activation: {self._activation}\nweight: {self._weight}"


class QuantConfig:
    def __init__(self, activation=None, weight=None):
        self._global = SingleLayerConfig(activation, weight) if (activation or weight) else None
        self._layer2config = {}
        self._prefix2config = {}
        self._type2config = {}
        self._qat_layer_mapping = {Linear: QuantedLinear, Conv2D: QuantedConv2D}
        self._customized_leaves = []

    def add_layer_config(self, layer, activation=None, weight=None):
        for lyr in (layer if isinstance(layer, (list, tuple)) else [layer]):
            self._layer2config[id(lyr)] = SingleLayerConfig(activation, weight)

    def add_name_config(self, layer_name, activation=None, weight=None):
        for n in (layer_name if isinstance(layer_name, (list, tuple)) else [layer_name]):
            self._prefix2config[n] = SingleLayerConfig(activation, weight)

    def add_type_config(self, layer_type, activation=None, weight=None):
        for t in (layer_type if isinstance(layer_type, (list, tuple)) else [layer_type]):
            self._type2config[t] = SingleLayerConfig(activation, weight)

    def add_qat_layer_mapping(self, source, target):
        self._qat_layer_mapping[source] = target

    def add_customized_leaf(self, layer_type):
        self._customized_leaves.append(layer_type)

    @property
    def customized_leaves(self):
        return self._customized_leaves

    @property
    def qat_layer_mappings(self):
        return self._qat_layer_mapping

    @property
    def default_qat_layer_mapping(self):
        return {Linear: QuantedLinear, Conv2D: QuantedConv2D}

    @property
    def global_config(self):
        return self._global

    def _get_config_by_layer(self, layer, name=''):
        if id(layer) in self._layer2config:
            return self._layer2config[id(layer)]
        for prefix, cfg in self._prefix2config.items():
            if name.startswith(prefix):
                return cfg
        for t, cfg in self._type2config.items():
            if isinstance(layer, t):
                return cfg
        return self._global

    def details(self):
        return str(self._global)

    def __str__(self):
        return self.details()


# ----------------------------------------------------------------- quanted layers
class _Quanted(Layer):
    def __init__(self, layer, q_config):
        super().__init__()
        self._inner = layer
        self.weight = layer.weight
        self.bias = getattr(layer, 'bias', None)
        self.weight_quanter = q_config.weight._instance(layer) if q_config and q_config.weight else None
        self.activation_quanter = q_config.activation._instance(layer) if q_config and q_config.activation else None

    def _qw(self):
        return self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight

    def _qx(self, x):
        return self.activation_quanter(x) if self.activation_quanter is not None else x


class QuantedLinear(_Quanted):
    def forward(self, x):
        from ..nn import functional as F
        return F.linear(self._qx(x), self._qw(), self.bias)


class QuantedConv2D(_Quanted):
    def forward(self, x):
        from ..nn import functional as F
        c = self._inner
        return F.conv2d(self._qx(x), self._qw(), self.bias, c._stride, c._padding, c._dilation, c._groups,
                        c._data_format)


class ObserveWrapper(Layer):
    """PTQ wrapper observing a leaf layer's input (activation) and weight."""

    def __init__(self, observer, observed, observe_input=True):
        super().__init__()
        self._observer = observer
        self._observed = observed
        self._observe_input = observe_input

    def forward(self, *inputs, **kw):
        if self._observe_input:
            inputs = (self._observer(inputs[0]),) + tuple(inputs[1:])
        return self._observed(*inputs, **kw)


# ----------------------------------------------------------------- passes
class Quantization(metaclass=abc.ABCMeta):
    def __init__(self, config):
        self._config = copy.deepcopy(config) if config is not None else QuantConfig()

    @abc.abstractmethod
    def quantize(self, model, inplace=False):
        pass

    def convert(self, model, inplace=False, remain_weight=False, to_fp8=False):
        """Freezes quanters/observers into fixed quant-dequant ops (or fp8 GEMMs)."""
        _model = model if inplace else copy.deepcopy(model)
        self._convert(_model, to_fp8)
        return _model

    def _convert(self, layer, to_fp8):
        for name, sub in list(layer._sub_layers.items()):
            if isinstance(sub, _Quanted):
                act_scale = sub.activation_quanter.scales() if sub.activation_quanter is not None else None
                if to_fp8 and isinstance(sub, QuantedLinear):
                    layer._sub_layers[name] = FP8Linear(sub._inner, act_scale)
                    continue
                if sub.weight_quanter is not None:
                    w = sub.weight_quanter(sub.weight)
                    with torch.no_grad():
                        sub._inner.weight._t.copy_(_unwrap(w))
                frozen = sub._inner
                if act_scale is not None:
                    frozen = _Sequential2(LinearQuanterDequanter(act_scale, sub.activation_quanter.bit_length()),
                                          sub._inner)
                layer._sub_layers[name] = frozen
            elif isinstance(sub, ObserveWrapper):
                s = sub._observer.cal_thresholds()
                if to_fp8 and isinstance(sub._observed, Linear):
                    layer._sub_layers[name] = FP8Linear(sub._observed, s)
                else:
                    layer._sub_layers[name] = _Sequential2(LinearQuanterDequanter(s, sub._observer.bit_length()),
                                                           sub._observed)
            else:
                self._convert(sub, to_fp8)

    def _is_leaf(self, layer):
        return not layer._sub_layers or any(isinstance(layer, t) for t in self._config.customized_leaves)


class _Sequential2(Layer):
    def __init__(self, a, b):
        super().__init__()
        self.quanter = a
        self.layer = b

    def forward(self, x, *rest, **kw):
        return self.layer(self.quanter(x), *rest, **kw)


class FP8Linear(Layer):
    """Linear on e4m3 operands with per-tensor scales.  On MI355X the weight is quantised (once,
    for frozen eval-mode weights) into the [out, in] e4m3 image the hand-written fp8 MFMA kernel reads
    (ops.gemm.hip_fp8_mm; scales stay on the device) and activations are quantised per call;
    elsewhere a dequantised-matmul emulation of the same numerics."""

    def __init__(self, linear, act_absmax=None):
        super().__init__()
        self.weight = linear.weight
        self.bias = linear.bias
        self._act_absmax = float(_unwrap(act_absmax).max()) if act_absmax is not None else None
        self._wq = None  # (weight version, data_ptr, e4m3 [out, in], scale)

    def _quant_weight(self, w):
        # cached only for frozen weights in eval mode: fused optimizer kernels update parameters
        # in place without bumping the version counter, so a trainable weight is re-quantised
        key = (w._version, w.data_ptr())
        frozen = not self.training and not w.requires_grad
        if self._wq is None or self._wq[0] != key or not frozen:
            from ..ops.gemm import fp8_quantize
            q, s = fp8_quantize(w.detach().t())
            self._wq = (key, q.contiguous(), s)
        return self._wq[1], self._wq[2]

    def forward(self, x):
        from .. import ops
        t = _unwrap(x)
        w = self.weight._t
        if ops.use_hip(t):
            t2 = t.reshape(-1, t.shape[-1])
            if self._act_absmax is not None:
                sx = torch.full((1,), self._act_absmax / 448.0, device=t.device)
                xq = (t2.float() / sx).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
            else:
                xq, sx = ops.gemm.fp8_quantize(t2)
            wq, sw = self._quant_weight(w)
            if t.dtype == torch.bfloat16 and ops.gemm.hip_fp8_ok(xq, wq):
                b = self.bias._t if self.bias is not None else None
                out = ops.gemm.hip_fp8_mm(xq, wq, scale_a=sx, scale_b=sw,
                                          bias=None if b is None else b.to(torch.bfloat16).contiguous())
                return _wrap(out.reshape(*t.shape[:-1], out.shape[-1]))
            out = ops.gemm.fp8_gemm(t, w, bias=None if self.bias is None else self.bias._t,
                                    output_dtype=str(t.dtype).replace('torch.', ''))
            return _wrap(out)
        fmax = 448.0
        sx = (self._act_absmax or float(t.abs().max())) / fmax
        sw = float(w.abs().max()) / fmax
        xq = (t / sx).clamp(-fmax, fmax).to(torch.float8_e4m3fn).to(t.dtype) * sx
        wq = (w / sw).clamp(-fmax, fmax).to(torch.float8_e4m3fn).to(w.dtype) * sw
        out = xq @ wq
        if self.bias is not None:
            out = out + self.bias._t
        return _wrap(out)


class QAT(Quantization):
    def quantize(self, model, inplace=False):
        if not model.training:
            raise ValueError("QAT expects a model in training mode")
        _model = model if inplace else copy.deepcopy(model)
        self._apply(_model, '')
        return _model

    def _apply(self, layer, prefix):
        mapping = self._config.qat_layer_mappings
        for name, sub in list(layer._sub_layers.items()):
            full = f"{prefix}.{name}" if prefix else name
            cfg = self._config._get_config_by_layer(sub, full)
            tgt = next((mapping[t] for t in mapping if type(sub) is t), None)
            if tgt is not None and cfg is not None:
                layer._sub_layers[name] = tgt(sub, cfg)
            else:
                self._apply(sub, full)


class PTQ(Quantization):
    def quantize(self, model, inplace=False):
        _model = model if inplace else copy.deepcopy(model)
        _model.eval()
        self._apply(_model, '')
        return _model

    def _apply(self, layer, prefix):
        for name, sub in list(layer._sub_layers.items()):
            full = f"{prefix}.{name}" if prefix else name
            cfg = self._config._get_config_by_layer(sub, full)
            if cfg is not None and self._is_leaf(sub) and cfg.activation is not None:
                layer._sub_layers[name] = ObserveWrapper(cfg.activation._instance(sub), sub)
            else:
                self._apply(sub, full)


__all__ = ["QuantConfig", "BaseQuanter", "BaseObserver", "quanter", "QAT", "PTQ"]

_ = (Tensor, Conv1D, Conv3D)
