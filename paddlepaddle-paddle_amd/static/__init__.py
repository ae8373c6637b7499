"""paddle.static (reference: python/paddle/static/__init__.py).  See program.py for the design."""
import contextlib

import torch

from .program import (Program, Block, program_guard, default_main_program, default_startup_program, data,  # noqa: F401
                      InputSpec, name_scope, append_backward, gradients, Ref, Const)
from .executor import (Executor, ParallelExecutor, global_scope, scope_guard, Scope, BuildStrategy,  # noqa: F401
                       ExecutionStrategy, CompiledProgram)
from .io import (save_inference_model, load_inference_model, serialize_program, serialize_persistables,  # noqa: F401
                 deserialize_program, deserialize_persistables, save, load, load_program_state,
                 set_program_state)
from . import nn  # noqa: F401
from . import amp  # noqa: F401
from .nn import py_func  # noqa: F401
from . import sequence as _sequence  # noqa: E402
from .sequence import create_lod_tensor  # noqa: F401
_sequence.install_tensor_methods()  # Tensor.set_lod / lod / (set_)recursive_sequence_lengths
from ..core.tensor import Tensor as Variable  # noqa: F401
from ..framework.param_attr import ParamAttr, WeightNormParamAttr  # noqa: F401


def save_to_file(path, content):
    with open(path, 'wb') as f:
        f.write(content)


def load_from_file(path):
    with open(path, 'rb') as f:
        return f.read()


def normalize_program(program, feed_vars, fetch_vars, **kw):
    return program.clone(for_test=True)


def cpu_places(device_count=None):
    from ..core.place import CPUPlace
    return [CPUPlace()] * (device_count or 1)


def cuda_places(device_ids=None):
    from ..core.place import CUDAPlace
    if device_ids is None:
        device_ids = list(range(torch.cuda.device_count()))
    return [CUDAPlace(i) for i in device_ids]


def xpu_places(device_ids=None):
    return []


@contextlib.contextmanager
def device_guard(device=None):
    """Ops recorded inside run on pipeline stage N for ``'gpu:N'`` (reference
    static.device_guard + the fleet pipeline optimizer's program split by op device); 'cpu' /
    None leave the stage unchanged.  Execution placement itself is the Executor's place."""
    from .program import _STAGE
    prev = _STAGE[0]
    if isinstance(device, str) and ':' in device:
        try:
            _STAGE[0] = int(device.split(':')[1])
        except ValueError:
            pass
    try:
        yield
    finally:
        _STAGE[0] = prev


@contextlib.contextmanager
def ipu_shard_guard(index=-1, stage=-1):
    yield


def set_ipu_shard(call_func, index=-1, stage=-1):
    return call_func


class IpuStrategy:
    def __init__(self):
        raise RuntimeError("IPU is not available on this framework (MI355X only)")


IpuCompiledProgram = IpuStrategy


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..nn.layer.layers import Layer
    return Layer().create_parameter(shape, attr=attr, dtype=dtype, is_bias=is_bias,
                                    default_initializer=default_initializer)


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    from ..tensor.creation import full
    t = full(shape, value, dtype)
    t.persistable = persistable
    if name:
        t._name = name
    return t


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True, print_tensor_type=True,  # noqa: A002,N802
          print_tensor_shape=True, print_tensor_lod=True, print_phase='both'):
    def show(x):
        print(message or '', x)
        return x
    from .program import recording
    if recording() and input._t.is_meta:
        return nn.py_func(show, input, input)
    show(input)
    return input


def accuracy(input, label, k=1, correct=None, total=None):  # noqa: A002
    from ..metric import accuracy as acc
    return acc(input, label, k)


def _persistent(shape, like):
    """A persistable fp32 accumulator on the program's device: recorded static ops update it in
    place on every Executor run (reference: create_global_variable(persistable=True))."""
    import torch
    from .program import _paused
    with _paused():
        dev = like.device if not like.is_meta else torch.device(_current_device())
        return torch.zeros(shape, dtype=torch.float32, device=dev)


def _current_device():
    from ..core.place import to_device
    from ..device import get_device
    return to_device(get_device())


class _force_record:
    """Ops whose only tensor inputs are these persistent accumulators are still recorded as program
    nodes (they must run on every Executor.run, not once while the program is built)."""

    def __init__(self, *ts):
        from .program import default_main_program
        self.prog = default_main_program()
        self.ids = {id(t) for t in ts}

    def __enter__(self):
        self.old = getattr(self.prog, '_force_record_ids', None)
        self.prog._force_record_ids = set(self.old or ()) | self.ids

    def __exit__(self, *exc):
        self.prog._force_record_ids = self.old
        return False


def _roc_auc(pos, neg):
    """Area under the ROC curve from per-threshold histograms (thresholds high -> low), the
    reference auc kernel's trapezoid sum, as tensor ops."""
    import torch
    tp = torch.cumsum(torch.flip(pos, [0]), 0)
    fp = torch.cumsum(torch.flip(neg, [0]), 0)
    tp0 = torch.cat([torch.zeros_like(tp[:1]), tp[:-1]])
    fp0 = torch.cat([torch.zeros_like(fp[:1]), fp[:-1]])
    area = ((fp - fp0) * (tp + tp0) * 0.5).sum()
    den = tp[-1] * fp[-1]
    return torch.where(den > 0, area / torch.where(den > 0, den, torch.ones_like(den)), torch.zeros_like(den))


def auc(input, label, curve='ROC', num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1, ins_tag_weight=None):  # noqa: A002
    """Streaming ROC AUC (reference static/nn/metric.py auc): positive-class scores are bucketed
    into ``num_thresholds + 1`` histograms; ``stat_pos`` / ``stat_neg`` accumulate over every run
    of the program (global AUC), a ring of the last ``slide_steps`` batches gives the batch AUC
    (``slide_steps = 0``: all steps).  Returns (auc_out, batch_auc_out,
    [batch_stat_pos, batch_stat_neg, stat_pos, stat_neg])."""
    import torch
    from ..core.tensor import _wrap, _unwrap
    if curve != 'ROC':
        raise ValueError("static auc computes the ROC curve (use paddle.metric.Auc(curve='PR') for PR)")
    T = int(num_thresholds)
    p, lab = _unwrap(input), _unwrap(label)
    pos_prob = p[:, 1] if (p.dim() == 2 and p.shape[1] == 2) else p.reshape([-1])
    idx = torch.clamp((pos_prob * T).to(torch.int64), 0, T)
    lf = lab.reshape([-1]).to(torch.float32)
    w = _unwrap(ins_tag_weight).reshape([-1]).to(torch.float32) if ins_tag_weight is not None else None
    pw = lf * w if w is not None else lf
    nw = (1.0 - lf) * w if w is not None else 1.0 - lf
    steps = max(int(slide_steps), 1)
    stat_pos, stat_neg = _persistent([T + 1], p), _persistent([T + 1], p)
    ring_pos, ring_neg = _persistent([steps, T + 1], p), _persistent([steps, T + 1], p)
    zeros = torch.zeros(T + 1, dtype=torch.float32, device=stat_pos.device)
    bpos = zeros.scatter_add(0, idx, pw)
    bneg = zeros.scatter_add(0, idx, nw)
    with _force_record(stat_pos, stat_neg, ring_pos, ring_neg):
        stat_pos.add_(bpos)
        stat_neg.add_(bneg)
        if int(slide_steps) == 0:
            batch_pos, batch_neg = stat_pos, stat_neg
        else:  # shift the ring by one batch and put this batch last
            ring_pos.copy_(torch.cat([ring_pos[1:], bpos.reshape([1, -1])], 0))
            ring_neg.copy_(torch.cat([ring_neg[1:], bneg.reshape([1, -1])], 0))
            batch_pos, batch_neg = ring_pos.sum(0), ring_neg.sum(0)
        auc_out = _roc_auc(stat_pos, stat_neg)
        batch_auc = _roc_auc(batch_pos, batch_neg)
    return _wrap(auc_out), _wrap(batch_auc), [_wrap(batch_pos), _wrap(batch_neg), _wrap(stat_pos), _wrap(stat_neg)]


def ctr_metric_bundle(input, label, ins_tag_weight=None):  # noqa: A002
    """CTR metric accumulators (reference static/nn/metric.py ctr_metric_bundle): persistable sums of
    squared error, absolute error, predicted ctr, q (sum of sigmoid(pred)), positives and
    instances over every run; MAE / RMSE / predicted ctr / q follow by dividing by the instance
    count.  ``ins_tag_weight`` (0/1 per instance) masks instances out.  Returns
    (local_sqrerr, local_abserr, local_prob, local_q, local_pos_num, local_ins_num)."""
    import torch
    from ..core.tensor import _wrap, _unwrap
    p, lab = _unwrap(input), _unwrap(label)
    x = p.reshape([-1]).to(torch.float32)
    y = lab.reshape([-1]).to(torch.float32)
    m = _unwrap(ins_tag_weight).reshape([-1]).to(torch.float32) if ins_tag_weight is not None else None
    acc = [_persistent([1], p) for _ in range(6)]
    d = x - y
    terms = [d * d, d.abs(), x, torch.sigmoid(x), y, torch.ones_like(x)]
    if m is not None:
        terms = [t * m for t in terms]
    with _force_record(*acc):
        for a, t in zip(acc, terms):
            a.add_(t.sum().reshape([1]))
    return tuple(_wrap(a) for a in acc)


class ExponentialMovingAverage:
    """EMA of parameters (reference: static/nn/common.py ExponentialMovingAverage): ``update()``
    after each step, ``apply()`` context swaps EMA weights in, ``restore()`` swaps back."""

    def __init__(self, decay=0.999, thres_steps=None, name=None):
        self.decay = decay
        self._ema = {}
        self._backup = {}
        self._step = 0

    def _params(self):
        return [p for p in default_main_program().all_parameters() if not p.stop_gradient] or \
            list(self._ema_params) if hasattr(self, '_ema_params') else \
            [p for p in default_main_program().all_parameters() if not p.stop_gradient]

    def update(self, parameters=None):
        self._step += 1
        ps = parameters if parameters is not None else self._params()
        self._ema_params = ps
        d = min(self.decay, (1 + self._step) / (10 + self._step))
        with torch.no_grad():
            for p in ps:
                e = self._ema.get(id(p))
                if e is None:
                    self._ema[id(p)] = p._t.detach().clone()
                else:
                    e.mul_(d).add_(p._t.detach(), alpha=1 - d)

    @contextlib.contextmanager
    def apply(self, executor=None, need_restore=True):
        with torch.no_grad():
            for p in getattr(self, '_ema_params', []):
                self._backup[id(p)] = p._t.detach().clone()
                p._t.copy_(self._ema[id(p)])
        try:
            yield
        finally:
            if need_restore:
                self.restore()

    def restore(self, executor=None):
        with torch.no_grad():
            for p in getattr(self, '_ema_params', []):
                if id(p) in self._backup:
                    p._t.copy_(self._backup.pop(id(p)))


