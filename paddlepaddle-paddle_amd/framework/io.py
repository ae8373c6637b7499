"""paddle.save / paddle.load (reference: python/paddle/framework/io.py:743 save, :985 load).

File format is the reference's: a pickle (protocol 2–4) in which every Tensor is reduced to
``(name, ndarray)`` (bf16 as uint16 arrays), so ``.pdparams`` / ``.pdopt`` files written here
load in the reference and vice versa.  Loading uses a RESTRICTED unpickler that only
resolves numpy array reconstruction and builtin containers — it never imports or calls
arbitrary code from the file.
"""
import collections
import copyreg
import io as _io
import os
import pickle

import numpy as np
import torch

from ..core.tensor import Tensor, Parameter, _wrap
from ..core.place import current_device

_SAFE = {
    ('numpy.core.multiarray', '_reconstruct'), ('numpy._core.multiarray', '_reconstruct'),
    ('numpy', 'ndarray'), ('numpy', 'dtype'), ('numpy.core.multiarray', 'scalar'),
    ('numpy._core.multiarray', 'scalar'), ('collections', 'OrderedDict'), ('builtins', 'tuple'),
    ('builtins', 'list'), ('builtins', 'dict'), ('builtins', 'set'), ('builtins', 'frozenset'),
    ('builtins', 'slice'), ('builtins', 'complex'), ('_codecs', 'encode'), ('numpy.core.numeric', '_frombuffer'),
    ('numpy._core.numeric', '_frombuffer'),
}


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _SAFE:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"paddle.load refuses to resolve {module}.{name} (not a tensor container)")


def _reduce_tensor(t):
    return (tuple, ((t.name, np.asarray(t) if t.dtype != torch.bfloat16 else t.numpy()),))


def _to_saveable(obj):
    if isinstance(obj, Tensor):
        return obj
    if isinstance(obj, torch.Tensor):
        return _wrap(obj)
    if isinstance(obj, collections.OrderedDict):
        return collections.OrderedDict((k, _to_saveable(v)) for k, v in obj.items())
    if isinstance(obj, dict):
        return {k: _to_saveable(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_saveable(v) for v in obj)
    from ..nn.layer.layers import Layer
    if isinstance(obj, Layer):
        raise ValueError("paddle do not support saving `paddle.nn.Layer` object.")
    return obj


def save(obj, path, protocol=4, **configs):
    if protocol < 2 or protocol > 4:
        raise ValueError(f"Expected 1<'protocol'<5, but received protocol={protocol}")
    obj = _to_saveable(obj)
    if isinstance(obj, dict) and obj and all(isinstance(v, Tensor) for v in obj.values()):
        # state_dict: record structured-name → parameter-name mapping like the reference
        obj = collections.OrderedDict(obj)
        obj['StructuredToParameterName@@'] = {k: v.name for k, v in obj.items() if isinstance(v, Tensor)}
    if isinstance(path, (str, os.PathLike)):
        d = os.path.dirname(os.fspath(path))
        if d:
            os.makedirs(d, exist_ok=True)
        f = open(path, 'wb')
        close = True
    else:
        f, close = path, False
    try:
        p = pickle.Pickler(f, protocol)
        p.dispatch_table = copyreg.dispatch_table.copy()
        p.dispatch_table[Tensor] = _reduce_tensor
        p.dispatch_table[Parameter] = _reduce_tensor
        p.dump(obj)
    finally:
        if close:
            f.close()


def _from_saved(v, return_numpy):
    if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str) and isinstance(v[1], np.ndarray):
        name, arr = v
        if return_numpy:
            return arr
        if arr.dtype == np.uint16:
            t = torch.from_numpy(arr.view(np.int16).copy()).view(torch.bfloat16)
        else:
            t = torch.from_numpy(np.ascontiguousarray(arr).copy())
        out = _wrap(t.to(current_device()))
        out.name = name
        return out
    if isinstance(v, np.ndarray):
        return v if return_numpy else _wrap(torch.from_numpy(v.copy()).to(current_device()))
    if isinstance(v, collections.OrderedDict):
        return collections.OrderedDict((k, _from_saved(x, return_numpy)) for k, x in v.items())
    if isinstance(v, dict):
        return {k: _from_saved(x, return_numpy) for k, x in v.items()}
    if isinstance(v, list):
        return [_from_saved(x, return_numpy) for x in v]
    if isinstance(v, tuple):
        return tuple(_from_saved(x, return_numpy) for x in v)
    return v


def load(path, **configs):
    return_numpy = configs.get('return_numpy', False)
    if isinstance(path, (str, os.PathLike)):
        with open(path, 'rb') as f:
            data = f.read()
    else:
        data = path.read()
    obj = _RestrictedUnpickler(_io.BytesIO(data), encoding='latin1').load()
    if isinstance(obj, dict):
        obj.pop('StructuredToParameterName@@', None)
        obj.pop('UnpackBigParamInfor@@', None)
    return _from_saved(obj, return_numpy)


def async_save(obj, path, protocol=4, sync_other_task=False, **configs):
    import threading
    snap = _to_saveable(obj)
    th = threading.Thread(target=save, args=(snap, path, protocol))
    th.start()
    return th
