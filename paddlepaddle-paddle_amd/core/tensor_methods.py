"""Attach the functional API as ``Tensor`` methods and operators.

Reference: python/paddle/tensor/__init__.py (``tensor_method_func``) and
python/paddle/base/dygraph/math_op_patch.py (operator overloading).
"""
import torch

from .tensor import Tensor, _wrap, _unwrap

_SKIP = {'to_tensor', 'meshgrid', 'arange', 'linspace', 'logspace',
         'eye', 'zeros', 'ones', 'empty', 'full', 'rand', 'randn', 'randint', 'randperm', 'uniform', 'normal',
         'standard_normal', 'gaussian', 'log_normal', 'tril_indices', 'triu_indices', 'fill_constant',
         'shape', 'numel', 'complex', 'hstack', 'vstack', 'dstack',
         'column_stack', 'row_stack', 'einsum', 'where', 'to_dlpack', 'assign'}
_KEEP_NATIVE = {'to', 'astype', 'cast', 'clone', 'detach', 'numpy', 'item', 'tolist', 'cpu', 'cuda', 'backward',
                'register_hook', 'contiguous', 'is_contiguous', 'dim', 'numel', 'fill_', 'zero_', 'copy_', 'apply',
                'apply_', 'set_value', 'is_floating_point', 'is_complex', 'is_integer', 'element_size', 'data_ptr'}


def _index(item):
    if isinstance(item, Tensor):
        t = item._t
        return t
    if isinstance(item, tuple):
        return tuple(_index(i) for i in item)
    if isinstance(item, list):
        if any(isinstance(i, Tensor) for i in item):
            return [_index(i) for i in item]
        return item
    return item


def _getitem(self, item):
    out = _wrap(self._t[_index(item)])
    sv = self.__dict__.get('_static_value')
    if sv is not None and isinstance(item, int):
        # a static-mode shape tensor (paddle.shape): its elements keep their record-time extents
        # (a dynamic dim's sentinel) for the shape inference of consumers such as reshape
        out.__dict__['_static_value'] = sv[item]
    return out


def _setitem(self, item, value):
    v = value._t if isinstance(value, Tensor) else value
    t = self._t
    if t.requires_grad and t.is_leaf:
        with torch.no_grad():
            t[_index(item)] = v
    else:
        t[_index(item)] = v


def _binop(fn):
    def op(self, other):
        o = other._t if isinstance(other, Tensor) else other
        return _wrap(fn(self._t, o))
    return op


def _rbinop(fn):
    def op(self, other):
        o = other._t if isinstance(other, Tensor) else other
        if not isinstance(o, torch.Tensor):
            o = torch.as_tensor(o, dtype=self._t.dtype if isinstance(o, (int, float)) and self._t.is_floating_point() else None,
                                device=self._t.device)
        return _wrap(fn(o, self._t))
    return op


def _ibinop(name):
    def op(self, other):
        o = other._t if isinstance(other, Tensor) else other
        getattr(self._t, name)(o)
        return self
    return op


def _truediv(a, b):
    return torch.true_divide(a, b)


def _matmul(a, b):
    return torch.matmul(a, b)


def install(namespace_funcs):
    T = Tensor
    for name, fn in namespace_funcs.items():
        if name in _SKIP or name in _KEEP_NATIVE or name.startswith('_'):
            continue
        if isinstance(getattr(T, name, None), property):
            continue
        setattr(T, name, fn)
    T.__getitem__ = _getitem
    T.__setitem__ = _setitem
    ops = {
        '__add__': torch.add, '__sub__': torch.sub, '__mul__': torch.mul, '__truediv__': _truediv,
        '__floordiv__': torch.floor_divide, '__mod__': torch.remainder, '__pow__': torch.pow,
        '__matmul__': _matmul, '__and__': torch.bitwise_and, '__or__': torch.bitwise_or,
        '__xor__': torch.bitwise_xor, '__lshift__': torch.bitwise_left_shift, '__rshift__': torch.bitwise_right_shift,
        '__eq__': torch.eq, '__ne__': torch.ne, '__lt__': torch.lt, '__le__': torch.le, '__gt__': torch.gt,
        '__ge__': torch.ge,
    }
    for k, f in ops.items():
        setattr(T, k, _binop(f))
    rops = {'__radd__': torch.add, '__rsub__': torch.sub, '__rmul__': torch.mul, '__rtruediv__': _truediv,
            '__rfloordiv__': torch.floor_divide, '__rmod__': torch.remainder, '__rpow__': torch.pow,
            '__rmatmul__': _matmul, '__rand__': torch.bitwise_and, '__ror__': torch.bitwise_or,
            '__rxor__': torch.bitwise_xor}
    for k, f in rops.items():
        setattr(T, k, _rbinop(f))
    iops = {'__iadd__': 'add_', '__isub__': 'sub_', '__imul__': 'mul_', '__itruediv__': 'div_',
            '__ifloordiv__': 'floor_divide_', '__imod__': 'remainder_', '__ipow__': 'pow_'}
    for k, m in iops.items():
        setattr(T, k, _ibinop(m))
    # `a @ b` goes through the AMP-tagged paddle.matmul (matmul_v2 is a white-list op)
    _mm = namespace_funcs['matmul']
    T.__matmul__ = lambda self, other: _mm(self, other if isinstance(other, Tensor) else _wrap(torch.as_tensor(other, device=self._t.device)))
    T.__rmatmul__ = lambda self, other: _mm(other if isinstance(other, Tensor) else _wrap(torch.as_tensor(other, device=self._t.device)), self)
    T.__neg__ = lambda self: _wrap(-self._t)
    T.__pos__ = lambda self: self
    T.__abs__ = lambda self: _wrap(self._t.abs())
    T.__invert__ = lambda self: _wrap(~self._t)
    T.__hash__ = lambda self: id(self)
    # torch-style conveniences that paddle also exposes on Tensor
    T.sum = namespace_funcs['sum']
    T.mean = namespace_funcs['mean']
    T.max = namespace_funcs['max']
    T.min = namespace_funcs['min']
    T.add_ = namespace_funcs['add_']
    T.subtract_ = namespace_funcs['subtract_']
    T.multiply_ = namespace_funcs['multiply_']
    T.scale_ = namespace_funcs['scale_']
    T.uniform_ = namespace_funcs['uniform_']
    T.normal_ = namespace_funcs['normal_']
    T.exponential_ = namespace_funcs['exponential_']
    T.expand = lambda self, *shape: namespace_funcs['expand'](self, shape[0] if len(shape) == 1 and isinstance(shape[0], (list, tuple)) else list(shape))
    T.reshape = lambda self, *shape, name=None: namespace_funcs['reshape'](self, shape[0] if len(shape) == 1 and isinstance(shape[0], (list, tuple, Tensor)) else list(shape))
    T.transpose = lambda self, perm, name=None: namespace_funcs['transpose'](self, perm)
    T.unbind = namespace_funcs['unbind']
    T.chunk = namespace_funcs['chunk']
    T.split = namespace_funcs['split']
    T.flatten = namespace_funcs['flatten']
    T.masked_fill = namespace_funcs['masked_fill']
    T.where = lambda self, x=None, y=None, name=None: namespace_funcs['where'](self, x, y)
    T.norm = namespace_funcs['norm']
    from .. import signal as _signal
    T.stft = _signal.stft
    T.istft = _signal.istft
