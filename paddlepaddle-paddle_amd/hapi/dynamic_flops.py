"""FLOPs counter (reference: python/paddle/hapi/dynamic_flops.py:28 flops, count_* rules):
forward hooks count multiply-adds per layer type on one synthetic batch."""
import numpy as np
import torch

from .. import nn
from ..core.tensor import Tensor


def _numel(t):
    return int(np.prod(t.shape)) if isinstance(t, Tensor) else 0


def count_convNd(m, x, y):  # noqa: N802
    k = int(np.prod(m.weight.shape[2:]))
    cin_per_group = m.weight.shape[1]
    bias = 1 if getattr(m, 'bias', None) is not None else 0
    m.total_ops += _numel(y) * (cin_per_group * k + bias)


def count_leaky_relu(m, x, y):
    m.total_ops += _numel(x[0])


def count_bn(m, x, y):
    n = _numel(x[0])
    m.total_ops += 2 * n if not m.training else 4 * n


def count_linear(m, x, y):
    m.total_ops += m.weight.shape[0] * _numel(y)


def count_avgpool(m, x, y):
    m.total_ops += _numel(y)


def count_adap_avgpool(m, x, y):
    kernel = np.array(x[0].shape[2:]) // np.array(y.shape[2:])
    m.total_ops += (int(np.prod(kernel)) + 1) * _numel(y)


def count_zero_ops(m, x, y):
    m.total_ops += 0


def count_parameters(m, x, y):
    m.total_params = sum(int(np.prod(p.shape)) for p in m.parameters())


_RULES = {
    nn.Conv1D: count_convNd, nn.Conv2D: count_convNd, nn.Conv3D: count_convNd,
    nn.Conv1DTranspose: count_convNd, nn.Conv2DTranspose: count_convNd, nn.Conv3DTranspose: count_convNd,
    nn.BatchNorm1D: count_bn, nn.BatchNorm2D: count_bn, nn.BatchNorm3D: count_bn, nn.BatchNorm: count_bn,
    nn.ReLU: count_zero_ops, nn.ReLU6: count_zero_ops, nn.LeakyReLU: count_leaky_relu, nn.Linear: count_linear,
    nn.Dropout: count_zero_ops, nn.AvgPool1D: count_avgpool, nn.AvgPool2D: count_avgpool, nn.AvgPool3D: count_avgpool,
    nn.AdaptiveAvgPool1D: count_adap_avgpool, nn.AdaptiveAvgPool2D: count_adap_avgpool,
    nn.AdaptiveAvgPool3D: count_adap_avgpool,
}


def flops(net, input_size, custom_ops=None, print_detail=False):
    from .model_summary import _make_inputs
    from ..core.place import current_device
    rules = dict(_RULES)
    rules.update(custom_ops or {})
    hooks = []
    layers = []
    for m in net.sublayers(include_self=True):
        if m._sub_layers and type(m) not in rules:
            continue
        m.total_ops = 0
        m.total_params = sum(int(np.prod(p.shape)) for p in m._parameters.values() if p is not None)
        fn = rules.get(type(m))
        if fn is None:
            continue
        layers.append(m)
        hooks.append(m.register_forward_post_hook(lambda lyr, inp, out, f=fn: f(lyr, inp, out)))
    was = net.training
    net.eval()
    try:
        with torch.no_grad():
            net(*_make_inputs(tuple(input_size), None, current_device()))
    finally:
        for h in hooks:
            h.remove()
        if was:
            net.train()
    total = sum(int(m.total_ops) for m in layers)
    if print_detail:
        for m in layers:
            print(f"{type(m).__name__:<24} ops {int(m.total_ops):>14,}  params {m.total_params:>12,}")
    print(f"Total Flops: {total}     Total Params: {sum(int(np.prod(p.shape)) for p in net.parameters())}")
    return total
