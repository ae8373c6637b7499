"""Automatic SParsity, n:m structured (reference: python/paddle/incubate/asp/ — prune_model,
decorate, calculate_density, set_excluded_layers, utils mask algorithms).

2:4 is the pattern CDNA4's sparse MFMA (``v_smfmac``) consumes: in every group of 4 weights along
the input dim, 2 are kept.  ``prune_model`` computes masks (magnitude, 1-D groups) and applies
them; ``decorate(optimizer)`` re-applies the masks after every step so pruned weights stay 0.
"""
import re

import numpy as np
import torch

from ..core.tensor import _unwrap

_excluded = set()
_masks = {}
# layer-type name (snake case) -> pruning function (weight ndarray, m, n, mask_algo, param_name)
# -> (pruned weight, mask); reference incubate/asp/supported_layer_list.py
_custom_prune = {}


def _snake(name):
    return re.sub(r'(?<!^)(?=[A-Z])', '_', name).lower()


def add_supported_layer(layer, pruning_func=None):
    """Register a layer (name, Layer instance or Layer class) whose parameters ``prune_model``
    prunes with ``pruning_func(weight_ndarray, m, n, mask_algo, param_name) -> (weight, mask)``
    (the built-in n:m magnitude mask when None)."""
    from ..nn.layer.layers import Layer
    if isinstance(layer, str):
        name = layer
    elif isinstance(layer, Layer):
        name = _snake(type(layer).__name__)
    elif isinstance(layer, type) and issubclass(layer, Layer):
        name = _snake(layer.__name__)
    else:
        raise TypeError(f"add_supported_layer expects a name or a Layer, got {type(layer)}")
    _custom_prune[name] = pruning_func


def calculate_density(x):
    t = _unwrap(x) if not isinstance(x, torch.Tensor) else x
    return float((t != 0).sum()) / max(t.numel(), 1)


def set_excluded_layers(param_names=None, main_program=None):
    _excluded.update(param_names or [])


def reset_excluded_layers(main_program=None):
    _excluded.clear()


def create_mask(w, n=2, m=4):
    """Keep the n largest |w| of every m consecutive weights along the last (input) dim."""
    t = w.detach()
    shape = t.shape
    flat = t.reshape(-1, shape[-1])
    pad = (-flat.shape[1]) % m
    if pad:
        flat = torch.nn.functional.pad(flat, (0, pad))
    g = flat.reshape(flat.shape[0], -1, m).abs()
    idx = g.topk(n, dim=-1).indices
    mask = torch.zeros_like(g, dtype=torch.bool).scatter_(-1, idx, True)
    mask = mask.reshape(flat.shape[0], -1)[:, :shape[-1]]
    return mask.reshape(shape)


def check_sparsity(w, n=2, m=4):
    t = _unwrap(w) if not isinstance(w, torch.Tensor) else w
    flat = t.reshape(-1, t.shape[-1])
    pad = (-flat.shape[1]) % m
    if pad:
        flat = torch.nn.functional.pad(flat, (0, pad))
    return bool(((flat.reshape(flat.shape[0], -1, m) != 0).sum(-1) <= n).all())


def _supported(name, p):
    return p.ndim >= 2 and name not in _excluded and not any(name.startswith(e) for e in _excluded)


def prune_model(model, n=2, m=4, mask_algo='mask_1d', with_mask=True):
    """Applies n:m masks to every eligible weight (Linear [in, out] is pruned along ``in``)."""
    out = {}
    owner = {}
    for lname, layer in model.named_sublayers(include_self=True):
        for pname, p in layer.named_parameters(include_sublayers=False):
            owner[id(p)] = _snake(type(layer).__name__)
    for name, p in model.named_parameters():
        if not _supported(name, p):
            continue
        t = _unwrap(p)
        fn = _custom_prune.get(owner.get(id(p), ''))
        if fn is not None:  # registered custom pruning function
            w_np, mask_np = fn(t.detach().float().cpu().numpy(), m, n, mask_algo, name)
            mask = torch.as_tensor(np.asarray(mask_np), device=t.device)
            with torch.no_grad():
                t.copy_(torch.as_tensor(np.asarray(w_np), device=t.device).to(t.dtype))
            if with_mask:
                _masks[id(p)] = (p, mask)
            out[name] = mask
            continue
        # paddle Linear weights are [in, out]: group along the input dim → transpose for masking
        w = t.t() if t.dim() == 2 else t
        mask = create_mask(w, n, m)
        mask = mask.t() if t.dim() == 2 else mask
        with torch.no_grad():
            t.mul_(mask.to(t.dtype))
        if with_mask:
            _masks[id(p)] = (p, mask)
        out[name] = mask
    return out


class _ASPOptimizer:
    def __init__(self, optimizer):
        self._inner = optimizer

    @torch.no_grad()
    def step(self):
        self._inner.step()
        for p, mask in _masks.values():
            _unwrap(p).mul_(mask.to(_unwrap(p).dtype))

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def __getattr__(self, n):
        return getattr(self._inner, n)


def decorate(optimizer):
    return _ASPOptimizer(optimizer)
