"""NaN/Inf debugging (reference: python/paddle/amp/debugging.py: TensorCheckerConfig,
enable_tensor_checker, check_numerics, check_layer_numerics)."""
import enum

import torch

from ..core.tensor import Tensor, _wrap, _unwrap


class DebugMode(enum.Enum):
    CHECK_NAN_INF_AND_ABORT = 0
    CHECK_NAN_INF = 1
    CHECK_ALL_FOR_OVERFLOW = 2
    CHECK_ALL = 3
    DUMP_ALL = 4


class TensorCheckerConfig:
    def __init__(self, enable, debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT, output_dir=None, checked_op_list=None,
                 skipped_op_list=None, debug_step=None, stack_height_limit=1):
        self.enable, self.debug_mode, self.output_dir = enable, debug_mode, output_dir
        self.checked_op_list, self.skipped_op_list = checked_op_list, skipped_op_list
        self.debug_step = debug_step


_checker = {'cfg': None, 'handles': []}


def check_numerics(tensor, op_type='', var_name='', debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT):
    t = _unwrap(tensor)
    if not t.is_floating_point():
        return _wrap(torch.zeros(3, dtype=torch.int64)), _wrap(torch.zeros(3))
    n_nan = int(torch.isnan(t).sum())
    n_inf = int(torch.isinf(t).sum())
    if (n_nan or n_inf) and debug_mode == DebugMode.CHECK_NAN_INF_AND_ABORT:
        raise RuntimeError(f"[check_numerics] op={op_type} var={var_name}: {n_nan} NaN, {n_inf} Inf")
    stats = torch.tensor([n_nan, n_inf, int((t == 0).sum())], dtype=torch.int64)
    vals = torch.stack([t.float().max(), t.float().min(), t.float().mean()]).cpu()
    return _wrap(stats), _wrap(vals)


def _hook(layer, inputs, outputs):
    outs = outputs if isinstance(outputs, (tuple, list)) else [outputs]
    for i, o in enumerate(outs):
        if isinstance(o, Tensor):
            check_numerics(o, type(layer).__name__, f"output_{i}", _checker['cfg'].debug_mode)


def enable_tensor_checker(checker_config, model=None):
    _checker['cfg'] = checker_config
    if model is not None and checker_config.enable:
        for l in model.sublayers(include_self=True):
            _checker['handles'].append(l.register_forward_post_hook(_hook))


def disable_tensor_checker():
    for h in _checker['handles']:
        h.remove()
    _checker['handles'].clear()
    _checker['cfg'] = None


def check_layer_numerics(func):
    def wrapper(self, *args, **kwargs):
        for i, a in enumerate(args):
            if isinstance(a, Tensor):
                check_numerics(a, type(self).__name__, f"input_{i}")
        out = func(self, *args, **kwargs)
        _hook(self, args, out) if _checker['cfg'] is not None else None
        return out
    return wrapper


def enable_operator_stats_collection():
    pass


def disable_operator_stats_collection():
    pass


def compare_accuracy(dump_path, another_dump_path, output_filename, loss_scale=1, dump_all_tensors=False):
    raise NotImplementedError("compare_accuracy: dump comparison not supported in this build")
