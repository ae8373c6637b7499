"""auto_cast / decorate (reference: python/paddle/amp/auto_cast.py:383 amp_guard, :696 amp_decorate, :901 auto_cast)."""
import contextlib

import torch

from ..core import dtype as _dt
from ..core.place import current_device

_state = {'enable': False, 'level': 'O0', 'dtype': torch.float16}


def _norm_layer_types():
    from ..nn.layer import norm as N
    return (N._BatchNormBase, N.LayerNorm, N.RMSNorm, N.GroupNorm, N.InstanceNorm1D)


@contextlib.contextmanager
def amp_guard(enable=True, custom_white_list=None, custom_black_list=None, level='O1', dtype='float16',
              use_promote=True):
    dt = _dt.to_torch_dtype(dtype)
    prev = dict(_state)
    _state.update(enable=enable, level=level, dtype=dt)
    dev = current_device().type
    try:
        if enable and level in ('O1', 'O2'):
            with torch.autocast(device_type=dev if dev == 'cuda' else 'cpu', dtype=dt):
                yield
        else:
            yield
    finally:
        _state.update(prev)


def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level='O1', dtype='float16',
              use_promote=True):
    return amp_guard(enable, custom_white_list, custom_black_list, level, dtype, use_promote)


def amp_state():
    return dict(_state)


def decorate(models, optimizers=None, level='O1', dtype='float16', master_weight=None, save_dtype=None,
             master_grad=False, excluded_layers=None):
    if level == 'O1':
        return (models, optimizers) if optimizers is not None else models
    dt = _dt.to_torch_dtype(dtype)
    single = not isinstance(models, (list, tuple))
    ms = [models] if single else list(models)
    excluded = tuple(_norm_layer_types())
    if excluded_layers is not None:
        extra = excluded_layers if isinstance(excluded_layers, (list, tuple)) else [excluded_layers]
        excluded = excluded + tuple(e for e in extra if isinstance(e, type))
    for m in ms:
        for layer in m.sublayers(include_self=True):
            if isinstance(layer, excluded):
                continue
            for n, p in layer._parameters.items():
                if p is not None and p._t.is_floating_point():
                    req = p._t.requires_grad
                    with torch.no_grad():
                        p._t = p._t.detach().to(dt).requires_grad_(req)
        m.__dict__['_casted_by_pure_fp16'] = True
    if optimizers is not None:
        opts = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
        for o in opts:
            o._multi_precision = True if master_weight is None else bool(master_weight)
    out_m = ms[0] if single else ms
    return (out_m, optimizers) if optimizers is not None else out_m


amp_decorate = decorate


def is_float16_supported(device=None):
    return torch.cuda.is_available()


def is_bfloat16_supported(device=None):
    return True
