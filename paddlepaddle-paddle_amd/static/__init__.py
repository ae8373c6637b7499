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
    yield


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


def auc(input, label, curve='ROC', num_thresholds=4095, topk=1, slide_steps=1, ins_tag_weight=None):  # noqa: A002
    from ..metric import Auc
    raise NotImplementedError("static auc op: use paddle.metric.Auc on fetched predictions")


def ctr_metric_bundle(input, label, ins_tag_weight=None):  # noqa: A002
    raise NotImplementedError("ctr_metric_bundle is a parameter-server metric (out of scope)")


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


