"""auto_cast / amp_guard / decorate.

Reference: python/paddle/amp/auto_cast.py:383 (``amp_guard``), :696 (``amp_decorate``), :901
(``auto_cast``), :1000 (``decorate``); the per-op cast rule lives in the eager tracer
(paddle/fluid/eager/amp_utils.h) and is applied here by ``core.amp_dispatch`` at the paddle op
boundary (every op named in a reference list is tagged with its reference op name).

* ``amp_guard(level='O1')``: white-list ops (matmul_v2 / conv2d / einsum / flash_attn /
  max_pool2d_with_index / fused rope) run in float16/bfloat16, black-list ops (softmax,
  layer_norm, reductions, exp/log/pow, losses, interp, embedding lookup, scatter) in float32,
  everything else follows type promotion.  ``custom_white_list``/``custom_black_list`` move ops
  between the lists (overlap is an error, like the reference).
* ``level='O2'``: pure low precision — only the extra black list (interp / lookup_table /
  scatter) stays float32.  ``level='OD'``: white list only.  ``O0`` / ``enable=False``: off.
* ``decorate(level='O2')``: casts parameters to the AMP dtype (normalisation layers and
  ``excluded_layers`` kept float32), enables optimizer master weights, ``master_grad``
  exposes float32 gradients, ``save_dtype`` casts ``state_dict`` values on save.
"""
import contextlib
import warnings

import torch

from ..core import dtype as _dt
from ..core import amp_dispatch as _disp
from ..core.place import current_device
from .amp_lists import _update_list
from ..core.tensor import register_param as _register_param

_state = {'enable': False, 'level': 'O0', 'dtype': torch.float16, 'use_promote': True}


def _norm_layer_types():
    from ..nn.layer import norm as N
    return (N._BatchNormBase, N.LayerNorm, N.RMSNorm, N.GroupNorm, N.InstanceNorm1D)


def _amp_dtype(dtype):
    d = str(dtype).lower().replace('paddle.', '').replace('torch.', '')
    if d not in ('float16', 'bfloat16'):
        raise ValueError("If enable amp, dtype should be 'float16' or 'bfloat16'.")
    return d


@contextlib.contextmanager
def amp_guard(enable=True, custom_white_list=None, custom_black_list=None, level='O1', dtype='float16',
              use_promote=True):
    level = str(level).upper()
    if level not in ('O0', 'OD', 'O1', 'O2'):
        raise ValueError("level should be O0, OD, O1 or O2.")
    d = _amp_dtype(dtype) if enable else (str(dtype).lower() if isinstance(dtype, str) else 'float16')
    if enable and current_device().type not in ('cuda', 'cpu'):
        warnings.warn(f"amp_guard on {current_device()} makes no effect")
    on = bool(enable) and level != 'O0'
    wl, bl = _update_list(custom_white_list, custom_black_list, level, d)
    st = _disp.STATE
    prev = (st.active, st.level, st.dtype, st.white, st.black, st.use_promote)
    prev_state = dict(_state)
    tdt = torch.bfloat16 if d == 'bfloat16' else torch.float16
    st.active, st.level, st.dtype = on, level, tdt
    st.white, st.black, st.use_promote = frozenset(wl), frozenset(bl), bool(use_promote)
    _state.update(enable=on, level=level if on else 'O0', dtype=tdt, use_promote=bool(use_promote))
    try:
        yield
    finally:
        st.active, st.level, st.dtype, st.white, st.black, st.use_promote = prev
        _state.clear()
        _state.update(prev_state)


def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level='O1', dtype='float16',
              use_promote=True):
    return amp_guard(enable, custom_white_list, custom_black_list, level, dtype, use_promote)


def amp_state():
    return dict(_state)


def _is_amp_enabled():
    return _disp.STATE.active


def _save_dtype_hook(dt):
    from ..core.tensor import Tensor, _wrap

    def hook(state):
        for k, v in list(state.items()):
            if isinstance(v, Tensor) and v._t.is_floating_point() and v._t.dtype != dt:
                state[k] = _wrap(v._t.detach().to(dt))
        return state
    return hook


def decorate(models, optimizers=None, level='O1', dtype='float16', master_weight=None, save_dtype=None,
             master_grad=False, excluded_layers=None):
    level = str(level).upper()
    if level not in ('O0', 'OD', 'O1', 'O2'):
        raise ValueError("level should be O0, OD, O1 or O2.")
    single = not isinstance(models, (list, tuple))
    ms = [models] if single else list(models)
    if save_dtype is not None:
        sd = str(save_dtype).lower().replace('paddle.', '')
        if sd not in ('float16', 'bfloat16', 'float32', 'float64'):
            raise ValueError(f"save_dtype must be float16/bfloat16/float32/float64, got {save_dtype}")
        for m in ms:
            m.register_state_dict_hook(_save_dtype_hook(_dt.to_torch_dtype(sd)))
    if level in ('O1', 'OD', 'O0'):
        return (models, optimizers) if optimizers is not None else models
    dt = _dt.to_torch_dtype(_amp_dtype(dtype))
    excluded_types = tuple(_norm_layer_types())
    excluded_objs = []
    if excluded_layers is not None:
        extra = excluded_layers if isinstance(excluded_layers, (list, tuple)) else [excluded_layers]
        excluded_types = excluded_types + tuple(e for e in extra if isinstance(e, type))
        excluded_objs = [e for e in extra if not isinstance(e, type)]
    skip = set()
    for e in excluded_objs:
        for l in e.sublayers(include_self=True):
            skip.add(id(l))
    for m in ms:
        for layer in m.sublayers(include_self=True):
            if isinstance(layer, excluded_types) or id(layer) in skip:
                continue
            for n, p in layer._parameters.items():
                if p is not None and p._t.is_floating_point():
                    req = p._t.requires_grad
                    with torch.no_grad():
                        p._t = p._t.detach().to(dt).requires_grad_(req)
                        _register_param(p)
                    if master_grad:
                        p.__dict__['_master_grad'] = True
        m.__dict__['_casted_by_pure_fp16'] = True
    if optimizers is not None:
        opts = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
        for o in opts:
            o._multi_precision = True if master_weight is None else bool(master_weight)
            if master_grad:
                o._master_grad = True
    out_m = ms[0] if single else ms
    return (out_m, optimizers) if optimizers is not None else out_m


amp_decorate = decorate


def is_float16_supported(device=None):
    return torch.cuda.is_available()


def is_bfloat16_supported(device=None):
    return True
