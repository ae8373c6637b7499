"""paddle.save / paddle.load (reference: python/paddle/framework/io.py:743 save, :985 load).

The file format is the reference's, in both of its shapes:

* a *state dict* (a dict whose values are all Tensors, or dicts holding none) is written the way
  ``_legacy_save`` (reference io.py:930) writes it: plain ndarray values (bf16 as uint16 arrays)
  plus the ``StructuredToParameterName@@`` name table, and with protocol 2/3 every array over
  2**30 bytes is split into ``key@@.i`` slices described by ``UnpackBigParamInfor@@``
  (reference io_utils.py:236 ``_unpack_saved_dict``);
* any other object is pickled with every Tensor reduced to ``(name, ndarray)``
  (reference io.py:383 ``_pickle_save``).

``load`` reassembles big-parameter slices (reference io_utils.py:218 ``_pack_loaded_dict``),
restores tensor names from the name table and converts ``(name, ndarray)`` tuples / bare
ndarrays like the reference's ``_parse_load_result`` (io.py:608).  Loading uses a RESTRICTED
unpickler that only resolves numpy array reconstruction and builtin containers — it never
imports or calls arbitrary code from the file.
"""
import collections
import copyreg
import io as _io
import math
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

NAME_TABLE = 'StructuredToParameterName@@'
UNPACK_INFO = 'UnpackBigParamInfor@@'


class _Refused(pickle.UnpicklingError, ValueError):
    """A pickle that names a callable outside the tensor-container allow-list."""


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _SAFE:
            return super().find_class(module, name)
        raise _Refused(f"paddle.load refuses to resolve {module}.{name} (not a tensor container)")


def _ndarray(t):
    """Host ndarray of a Tensor as the reference stores it (bf16 -> uint16 bit pattern)."""
    if isinstance(t, Tensor):
        t = t._t
    t = t.detach()
    if t.dtype == torch.bfloat16:
        return t.cpu().view(torch.int16).numpy().view(np.uint16)
    return t.cpu().numpy()


def _reduce_tensor(t):
    return (tuple, ((t.name, _ndarray(t)),))


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


def _contains(obj, cond):
    if cond(obj):
        return True
    if type(obj) in (dict, collections.OrderedDict):
        return any(_contains(v, cond) for v in obj.values())
    if type(obj) in (list, tuple):
        return any(_contains(v, cond) for v in obj)
    return False


def _is_state_dict(obj):
    """reference io.py:488: every value a Tensor, or a dict that holds no paddle object."""
    if not isinstance(obj, dict):
        return False
    from ..nn.layer.layers import Layer
    for v in obj.values():
        if isinstance(v, dict):
            if any(_contains(x, lambda o: isinstance(o, (Tensor, Layer))) for x in v.values()):
                return False
        elif not isinstance(v, Tensor):
            return False
    return True


def _build_saved_state_dict(state_dict):
    out, names = {}, {}
    for k, v in state_dict.items():
        if isinstance(v, Tensor):
            out[k] = _ndarray(v)
            names[k] = v.name
        else:
            out[k] = v
    out[NAME_TABLE] = names
    return out


def _unpack_saved_dict(saved, protocol, max_bytes=2 ** 30):
    """Split ndarrays over 2**30 bytes into ``key@@.i`` slices for pickle protocols 2/3."""
    if not (1 < protocol < 4) or not isinstance(saved, dict):
        return saved
    info = {}
    for key in list(saved.keys()):
        v = saved[key]
        if not isinstance(v, np.ndarray):
            continue
        cap = int((max_bytes - 1) / v.dtype.itemsize)
        n = int(np.prod(v.shape))
        if n <= cap:
            continue
        flat = v.reshape(-1)
        parts = []
        for i in range(int(math.ceil(n / cap))):
            name = f"{key}@@.{i}"
            parts.append(name)
            saved[name] = flat[i * cap:(i + 1) * cap]
        info[key] = {'OriginShape': v.shape, 'slices': parts}
        del saved[key]
    if info:
        saved[UNPACK_INFO] = info
    return saved


def _pack_loaded_dict(obj):
    if isinstance(obj, dict) and UNPACK_INFO in obj:
        info = obj.pop(UNPACK_INFO)
        for key, meta in info.items():
            obj[key] = np.concatenate([obj.pop(p) for p in meta['slices']]).reshape(meta['OriginShape'])
    return obj


def _open(path, mode):
    if isinstance(path, (str, os.PathLike)):
        if 'w' in mode:
            fn = os.path.basename(os.fspath(path))
            if fn == '':
                raise ValueError("The input path MUST be format of dirname/filename, but received filename is empty")
            d = os.path.dirname(os.fspath(path))
            if d:
                os.makedirs(d, exist_ok=True)
        return open(path, mode), True
    if not hasattr(path, 'write' if 'w' in mode else 'read'):
        raise ValueError(f"only supports saving objects to file and `BytesIO`, but got {type(path)}")
    return path, False


def save(obj, path, protocol=4, **configs):
    if not isinstance(protocol, int):
        raise ValueError(f"The 'protocol' MUST be `int`, but received {type(protocol)}")
    if protocol < 2 or protocol > 4:
        raise ValueError(f"Expected 1<'protocol'<5, but received protocol={protocol}")
    from ..static.program import Program
    if isinstance(obj, Program):
        from ..static.io import serialize_program
        f, close = _open(path, 'wb')
        try:
            f.write(serialize_program(list(obj.feeds.keys()), [], program=obj))
        finally:
            if close:
                f.close()
        return
    obj = _to_saveable(obj)
    f, close = _open(path, 'wb')
    try:
        if _is_state_dict(obj):
            pickle.dump(_unpack_saved_dict(_build_saved_state_dict(obj), protocol), f, protocol=protocol)
        else:
            p = pickle.Pickler(f, protocol)
            p.dispatch_table = copyreg.dispatch_table.copy()
            p.dispatch_table[Tensor] = _reduce_tensor
            p.dispatch_table[Parameter] = _reduce_tensor
            p.dump(obj)
    finally:
        if close:
            f.close()


def _to_tensor(arr, name=None):
    if arr.dtype == np.uint16:  # bf16 bit pattern
        t = torch.from_numpy(np.ascontiguousarray(arr).view(np.int16).copy()).view(torch.bfloat16)
    else:
        t = torch.from_numpy(np.ascontiguousarray(arr).copy())
    out = _wrap(t.to(current_device()))
    if name:
        out.name = name
    return out


def _is_name_tuple(v):
    return isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str) and isinstance(v[1], np.ndarray)


def _convert(v, cond, fn):
    if cond(v):
        return fn(v)
    if type(v) in (dict, collections.OrderedDict):
        return type(v)((k, _convert(x, cond, fn)) for k, x in v.items())
    if type(v) is list:
        return [_convert(x, cond, fn) for x in v]
    if type(v) is tuple:
        return tuple(_convert(x, cond, fn) for x in v)
    if type(v) is set:
        return {_convert(x, cond, fn) for x in v}
    return v


def _parse_load_result(obj, return_numpy):
    """(name, ndarray) tuples -> named Tensors if any exist, else every ndarray -> Tensor."""
    if _contains(obj, _is_name_tuple):
        return _convert(obj, _is_name_tuple, (lambda t: t[1]) if return_numpy else (lambda t: _to_tensor(t[1], t[0])))
    return _convert(obj, lambda v: isinstance(v, np.ndarray), (lambda a: a) if return_numpy else _to_tensor)


def load(path, **configs):
    return_numpy = configs.get('return_numpy', False)
    keep_names = configs.get('keep_name_table', False)
    if isinstance(path, (str, os.PathLike)):
        if os.path.isdir(path) or not os.path.exists(path):
            from ..static.io import load_persistables_dir
            return load_persistables_dir(path, **configs)
        with open(path, 'rb') as f:
            data = f.read()
    else:
        data = path.read()
    try:
        obj = _RestrictedUnpickler(_io.BytesIO(data), encoding='latin1').load()
    except _Refused:
        raise
    except (pickle.UnpicklingError, EOFError, ValueError, IndexError, KeyError) as e:
        # not a pickle: a serialized Program / binary tensor (static formats)
        from ..static.io import load_binary_object
        r = load_binary_object(data)
        if r is None:
            raise ValueError(f"`paddle.load` can not parse the file: {path} ({e})")
        return r
    if isinstance(obj, dict):
        obj = _pack_loaded_dict(obj)
        if NAME_TABLE in obj:
            names = obj[NAME_TABLE]
            for k, n in names.items():
                if isinstance(obj.get(k), np.ndarray):
                    obj[k] = obj[k] if return_numpy else _to_tensor(obj[k], n)
            if not keep_names:
                del obj[NAME_TABLE]
            return obj
    return _parse_load_result(obj, return_numpy)


def async_save(obj, path, protocol=4, sync_other_task=False, **configs):
    import threading
    snap = _to_saveable(obj)
    th = threading.Thread(target=save, args=(snap, path, protocol))
    th.start()
    return th
