"""NaN/Inf debugging, operator dtype statistics and fp32-vs-low-precision accuracy comparison.

Reference: python/paddle/amp/debugging.py (TensorCheckerConfig, enable_tensor_checker,
check_numerics, check_layer_numerics, enable/disable_operator_stats_collection,
collect_operator_stats, compare_accuracy) and python/paddle/amp/accuracy_compare.py (dump-line
format and the per-tensor fp32/fp16 comparison).

Ops tagged with their reference op name (``core.amp_dispatch.amp_op``) report their input
dtype to the operator-stats table and, while a tensor checker with ``output_dir`` is enabled,
dump one statistics line per floating output:

    [PRECISION] [device=gpu:0] op=matmul_v2, tensor=out_0, dtype=bfloat16, numel=4096, num_nan=0,
    num_inf=0, num_zero=3, max=1.25, min=-1.5, mean=0.01

``compare_accuracy`` pairs the lines of an fp32 run with those of a low-precision run (same
op/tensor key, in order) and writes a CSV report (the reference writes .xlsx through
xlsxwriter, which this image does not ship).
"""
import contextlib
import csv
import enum
import os

import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from ..core import amp_dispatch as _disp


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
        self.checked_op_list = set(checked_op_list) if checked_op_list else None
        self.skipped_op_list = set(skipped_op_list) if skipped_op_list else set()
        self.debug_step = debug_step
        self.stack_height_limit = stack_height_limit
        self.current_step_id = 0
        if debug_step is not None:
            if not (isinstance(debug_step, (list, tuple)) and len(debug_step) == 2 and debug_step[0] < debug_step[1]):
                raise ValueError("debug_step must be [start, end) with start < end")

    def update_and_check_step_id(self):
        self.current_step_id += 1
        if self.debug_step is None:
            return self.enable
        return self.enable and self.debug_step[0] <= self.current_step_id - 1 < self.debug_step[1]

    def start_check_nan_inf(self):
        pass

    def stop_check_nan_inf(self):
        pass


_checker = {'cfg': None, 'handles': [], 'file': None, 'active': False}


def _stats(t):
    f = t.detach().float()
    n_nan = int(torch.isnan(f).sum())
    n_inf = int(torch.isinf(f).sum())
    n_zero = int((f == 0).sum())
    fin = f[torch.isfinite(f)]
    if fin.numel():
        mx, mn, mean = float(fin.max()), float(fin.min()), float(fin.mean())
    else:
        mx = mn = mean = 0.0
    return n_nan, n_inf, n_zero, mx, mn, mean


def check_numerics(tensor, op_type='', var_name='', debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT):
    t = _unwrap(tensor)
    if not t.is_floating_point():
        return _wrap(torch.zeros(3, dtype=torch.int64)), _wrap(torch.zeros(3))
    n_nan, n_inf, n_zero, mx, mn, mean = _stats(t)
    if (n_nan or n_inf) and debug_mode == DebugMode.CHECK_NAN_INF_AND_ABORT:
        raise RuntimeError(f"[check_numerics] op={op_type} var={var_name}: {n_nan} NaN, {n_inf} Inf")
    return _wrap(torch.tensor([n_nan, n_inf, n_zero], dtype=torch.int64)), _wrap(torch.tensor([mx, mn, mean]))


_DT_NAME = {torch.float32: 'float32', torch.float16: 'float16', torch.bfloat16: 'bfloat16', torch.float64: 'float64'}


def _dump_line(op, name, t):
    n_nan, n_inf, n_zero, mx, mn, mean = _stats(t)
    dev = f"gpu:{t.device.index or 0}" if t.is_cuda else 'cpu'
    return (f"[PRECISION] [device={dev}] op={op}, tensor={name}, dtype={_DT_NAME.get(t.dtype, str(t.dtype))}, "
            f"numel={t.numel()}, num_nan={n_nan}, num_inf={n_inf}, num_zero={n_zero}, max={mx:.6e}, min={mn:.6e}, "
            f"mean={mean:.6e}")


def _op_post(op, out):
    cfg = _checker['cfg']
    if cfg is None or not _checker['active']:
        return
    if cfg.checked_op_list is not None and op not in cfg.checked_op_list:
        return
    if op in cfg.skipped_op_list:
        return
    outs = out if isinstance(out, (tuple, list)) else [out]
    for i, o in enumerate(outs):
        if not isinstance(o, Tensor) or not o._t.is_floating_point():
            continue
        if cfg.debug_mode == DebugMode.DUMP_ALL or cfg.output_dir:
            line = _dump_line(op, f"out_{i}", o._t)
            if _checker['file'] is not None:
                _checker['file'].write(line + '\n')
            else:
                print(line)
        if cfg.debug_mode in (DebugMode.CHECK_NAN_INF_AND_ABORT, DebugMode.CHECK_NAN_INF):
            check_numerics(o, op, f"out_{i}", cfg.debug_mode)


def _hook(layer, inputs, outputs):
    outs = outputs if isinstance(outputs, (tuple, list)) else [outputs]
    for i, o in enumerate(outs):
        if isinstance(o, Tensor):
            check_numerics(o, type(layer).__name__, f"output_{i}", _checker['cfg'].debug_mode)


def enable_tensor_checker(checker_config, model=None):
    """Turns the checker on for the current step (reference: call once per training step)."""
    cfg = checker_config
    _checker['cfg'] = cfg
    _checker['active'] = cfg.update_and_check_step_id()
    if not _checker['active']:
        return
    if cfg.output_dir and _checker['file'] is None:
        os.makedirs(cfg.output_dir, exist_ok=True)
        _checker['file'] = open(os.path.join(cfg.output_dir, f"worker_{os.getpid()}.log"), 'a')
    _disp.STATE.post = _op_post
    if model is not None:
        for l in model.sublayers(include_self=True):
            _checker['handles'].append(l.register_forward_post_hook(_hook))


def disable_tensor_checker():
    for h in _checker['handles']:
        h.remove()
    _checker['handles'].clear()
    _disp.STATE.post = None
    _checker['active'] = False
    if _checker['file'] is not None:
        _checker['file'].close()
        _checker['file'] = None
    _checker['cfg'] = None


def check_layer_numerics(func):
    def wrapper(self, *args, **kwargs):
        for i, a in enumerate(args):
            if isinstance(a, Tensor):
                check_numerics(a, type(self).__name__, f"input_{i}")
        out = func(self, *args, **kwargs)
        outs = out if isinstance(out, (tuple, list)) else [out]
        for i, o in enumerate(outs):
            if isinstance(o, Tensor):
                check_numerics(o, type(self).__name__, f"output_{i}")
        return out
    return wrapper


def set_checked_op_list(checked_op_list):
    if _checker['cfg'] is not None:
        _checker['cfg'].checked_op_list = set(checked_op_list)


def set_skipped_op_list(skipped_op_list):
    if _checker['cfg'] is not None:
        _checker['cfg'].skipped_op_list = set(skipped_op_list)


# ----------------------------------------------------------------------------- operator stats
def _print_operator_stats(op_count_dict):
    print("<{:-^120}>".format(" op list "))
    print("<{:-^40}".format(" Op Name "), "|", "{:-^17}".format(" FP16 Calls "), "|",
          "{:-^17}".format(" BF16 Calls "), "|", "{:-^17}".format(" FP32 Calls"), "|",
          "{:-^17}>".format(" Other Calls "))
    for op_type in sorted(op_count_dict or {}):
        c = op_count_dict[op_type]
        print("  %-40s|  %-17s|  %-17s|  %-17s|  %-17s" % (op_type, c[0], c[1], c[2], c[3]))
    print("<{:-^120}>\n".format(" op count: " + str(len(op_count_dict or {})) + " "))


def _stats_table():
    seen = _disp.STATE.ops_seen or {}
    return {op: [d.get('float16', 0), d.get('bfloat16', 0), d.get('float32', 0), d.get('other', 0)]
            for op, d in seen.items()}


def enable_operator_stats_collection():
    _disp.STATE.ops_seen = {}


def disable_operator_stats_collection():
    if _disp.STATE.ops_seen is None:
        return None
    table = _stats_table()
    _print_operator_stats(table)
    _disp.STATE.ops_seen = None
    return table


def get_operator_stats():
    return _stats_table()


@contextlib.contextmanager
def collect_operator_stats():
    enable_operator_stats_collection()
    try:
        yield
    finally:
        disable_operator_stats_collection()


# ----------------------------------------------------------------------------- accuracy compare
def _parse_line(line):
    if '[PRECISION]' not in line:
        return None
    info = {}
    for frag in line.strip().split(' '):
        w = frag.replace('[', '').replace(']', '').replace(',', '').split('=')
        if len(w) == 2:
            info[w[0]] = w[1]
    if 'op' not in info or 'tensor' not in info:
        return None
    for k in ('numel', 'num_nan', 'num_inf', 'num_zero'):
        info[k] = int(info.get(k, 0))
    for k in ('max', 'min', 'mean'):
        info[k] = float(info.get(k, 0.0))
    return info


def _parse_dir(path):
    out = []
    files = [path] if os.path.isfile(path) else sorted(os.path.join(path, f) for f in os.listdir(path))
    for fn in files:
        with open(fn) as fh:
            for line in fh:
                r = _parse_line(line)
                if r is not None:
                    out.append(r)
    return out


def compare_accuracy(dump_path, another_dump_path, output_filename, loss_scale=1, dump_all_tensors=False):
    """Compare an fp32 run's tensor dump with a low-precision run's (line order pairs same-key tensors).

    Writes ``output_filename`` (CSV; a ``.xlsx`` suffix is replaced by ``.csv``) with one row per
    paired tensor: key, both dtypes, max/min/mean of both, fp32/lowp mean ratio (``loss_scale``
    divided out of the low-precision side), inf/nan flags and an ``abnormal`` verdict.  Returns
    the number of abnormal rows.
    """
    a, b = _parse_dir(dump_path), _parse_dir(another_dump_path)
    by_key = {}
    for r in b:
        by_key.setdefault((r['op'], r['tensor']), []).append(r)
    rows, bad = [], 0
    for r in a:
        lst = by_key.get((r['op'], r['tensor']))
        if not lst:
            continue
        s = lst.pop(0)
        lowp_mean = s['mean'] / loss_scale if loss_scale else s['mean']
        ratio = r['mean'] / lowp_mean if lowp_mean != 0 else (1.0 if r['mean'] == 0 else np.inf)
        overflow = s['num_inf'] > 0 or s['num_nan'] > 0
        fp32_bad = r['num_inf'] > 0 or r['num_nan'] > 0
        # fp16 range / precision problems: overflow in low precision only, or a mean that drifts
        abnormal = (overflow and not fp32_bad) or not np.isclose(r['mean'], lowp_mean, rtol=5e-2, atol=1e-3)
        bad += int(abnormal)
        if dump_all_tensors or abnormal or overflow or fp32_bad:
            rows.append([f"{r['op']}/{r['tensor']}", r['dtype'], s['dtype'], r['numel'], r['max'], s['max'], r['min'],
                         s['min'], r['mean'], s['mean'], ratio, int(fp32_bad), int(overflow), int(abnormal)])
    if output_filename.endswith('.xlsx'):
        output_filename = output_filename[:-5] + '.csv'
    d = os.path.dirname(output_filename)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(output_filename, 'w', newline='') as fh:
        w = csv.writer(fh)
        w.writerow(['tensor', 'fp32_dtype', 'lowp_dtype', 'numel', 'fp32_max', 'lowp_max', 'fp32_min', 'lowp_min',
                    'fp32_mean', 'lowp_mean', 'fp32_div_lowp', 'fp32_inf_nan', 'lowp_inf_nan', 'abnormal'])
        w.writerows(rows)
    return bad
