"""paddle.nn.utils (reference: python/paddle/nn/utils/*.py)."""
import torch

from ..core.tensor import Tensor, Parameter, _wrap, _unwrap
from .clip import clip_grad_norm_, clip_grad_value_  # noqa: F401


def parameters_to_vector(parameters, name=None):
    return _wrap(torch.cat([p._t.reshape(-1) for p in parameters]))


def vector_to_parameters(vec, parameters, name=None):
    v = _unwrap(vec)
    off = 0
    with torch.no_grad():
        for p in parameters:
            n = p._t.numel()
            p._t.copy_(v[off:off + n].reshape(p._t.shape))
            off += n


def _norm_except_dim(w, dim):
    if dim == -1:
        return w.norm()
    dims = [i for i in range(w.dim()) if i != dim]
    return w.norm(dim=dims, keepdim=True)


def weight_norm(layer, name='weight', dim=0):
    w = getattr(layer, name)
    g = Parameter(_norm_except_dim(w._t.detach(), dim))
    v = Parameter(w._t.detach().clone())
    del layer._parameters[name]
    layer.add_parameter(name + '_g', g)
    layer.add_parameter(name + '_v', v)

    def hook(l, inputs):
        vv, gg = getattr(l, name + '_v')._t, getattr(l, name + '_g')._t
        object.__setattr__(l, name, _wrap(vv * (gg / _norm_except_dim(vv, dim))))
    hook(layer, None)
    layer._wn_hook = layer.register_forward_pre_hook(hook)
    return layer


def remove_weight_norm(layer, name='weight'):
    w = getattr(layer, name)
    layer._wn_hook.remove()
    del layer._parameters[name + '_g']
    del layer._parameters[name + '_v']
    layer.__dict__.pop(name, None)
    layer.add_parameter(name, Parameter(w._t.detach()))
    return layer


def spectral_norm(layer, name='weight', n_power_iterations=1, eps=1e-12, dim=None):
    from .layer.norm import SpectralNorm
    w = getattr(layer, name)
    dim = 0 if dim is None else dim
    sn = SpectralNorm(w.shape, dim, n_power_iterations, eps)
    orig = Parameter(w._t.detach().clone())
    del layer._parameters[name]
    layer.add_parameter(name + '_orig', orig)
    layer.add_sublayer(name + '_sn', sn)

    def hook(l, inputs):
        object.__setattr__(l, name, sn(getattr(l, name + '_orig')))
    hook(layer, None)
    layer.register_forward_pre_hook(hook)
    return layer
