"""paddle manipulation API (reference: python/paddle/tensor/manipulation.py)."""
import builtins

import numpy as np
import torch

from ._helpers import _w, _u, _t, _axis, _shape, _dtype, Tensor
from ..core.amp_dispatch import amp_op as _amp_op


def cast(x, dtype):
    return _w(_u(x).to(_dtype(dtype)))


def cast_(x, dtype):
    x._t = x._t.to(_dtype(dtype))
    return x


def _paddle_shape(t, shape):
    shape = _shape(shape)
    if 0 in shape:  # paddle: 0 = copy the input's dim at that position
        shape = [t.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return shape


def _is_var(v):
    return isinstance(v, Tensor) and v._t.is_meta


def _runtime_reshape(x, *dims):
    shp = []
    for d in dims:
        if isinstance(d, Tensor):
            shp.extend(int(v) for v in d._t.reshape(-1).tolist())
        else:
            shp.append(int(d))
    return _w(x._t.reshape(_paddle_shape(x._t, shp)))


def _static_reshape(x, shape):
    """reshape whose target shape holds static-mode tensors (paddle.shape results, their elements,
    a shape Variable): a recorded node that reads the extents at run time (the reference's
    ShapeTensor / ShapeTensorList inputs of reshape2).  The recorded output extents: each tensor
    element's record-time value (a dynamic dim's sentinel) when known, else -1."""
    from ..static.program import py_node
    t = _u(x)
    items = list(shape) if isinstance(shape, (list, tuple)) else [shape]
    rec = []
    for d in items:
        if isinstance(d, Tensor):
            sv = d.__dict__.get('_static_value')
            if sv is None:
                if d._t.dim() == 0 or d._t.numel() == 1:
                    rec.append(-1)
                else:
                    raise ValueError("reshape: a shape tensor needs its record-time extents (paddle.shape)")
            else:
                rec.extend(sv if isinstance(sv, (list, tuple)) else [sv])
        else:
            rec.append(int(d))
    meta = torch.empty(t.reshape(_paddle_shape(t, rec)).shape, dtype=t.dtype, device='meta')
    return py_node(_runtime_reshape, [x, *items], [meta])[0]


def reshape(x, shape, name=None):
    t = _u(x)
    if t.is_meta and (_is_var(shape) or (isinstance(shape, (list, tuple)) and any(_is_var(d) for d in shape))):
        return _static_reshape(x, shape)
    return _w(t.reshape(_paddle_shape(t, shape)))


def reshape_(x, shape, name=None):
    x._t = x._t.reshape(_paddle_shape(x._t, shape))
    return x


def view(x, shape_or_dtype, name=None):
    t = _u(x)
    if isinstance(shape_or_dtype, (list, tuple, Tensor)):
        return _w(t.view(_paddle_shape(t, shape_or_dtype)))
    return _w(t.view(_dtype(shape_or_dtype)))


def view_as(x, other, name=None):
    return _w(_u(x).view_as(_u(other)))


def as_strided(x, shape, stride, offset=0, name=None):
    return _w(torch.as_strided(_u(x), _shape(shape), list(stride), offset))


def transpose(x, perm, name=None):
    return _w(_u(x).permute(*[int(p) for p in perm]))


def transpose_(x, perm, name=None):
    x._t = x._t.permute(*perm).contiguous()
    return x


def t(input, name=None):  # noqa: A002
    tt = _u(input)
    return _w(tt.t() if tt.dim() == 2 else tt)


def t_(input, name=None):  # noqa: A002
    input._t = input._t.t() if input._t.dim() == 2 else input._t
    return input


def moveaxis(x, source, destination, name=None):
    return _w(torch.movedim(_u(x), source, destination))


def concat(x, axis=0, name=None):
    ts = [_u(e) for e in x]
    return _w(torch.cat(ts, dim=int(_u(axis)) if not isinstance(axis, int) else axis))


def stack(x, axis=0, name=None):
    return _w(torch.stack([_u(e) for e in x], dim=axis))


def hstack(x, name=None):
    return _w(torch.hstack([_u(e) for e in x]))


def vstack(x, name=None):
    return _w(torch.vstack([_u(e) for e in x]))


def dstack(x, name=None):
    return _w(torch.dstack([_u(e) for e in x]))


def column_stack(x, name=None):
    return _w(torch.column_stack([_u(e) for e in x]))


row_stack = vstack


def split(x, num_or_sections, axis=0, name=None):
    t = _u(x)
    axis = int(_u(axis)) if isinstance(axis, Tensor) else axis
    n = t.shape[axis]
    if isinstance(num_or_sections, int):
        if n % num_or_sections != 0:
            raise ValueError(f"split: dim {n} not divisible by {num_or_sections}")
        return [_w(p) for p in torch.split(t, n // num_or_sections, dim=axis)]
    secs = [int(_u(s)) if isinstance(s, Tensor) else int(s) for s in num_or_sections]
    if -1 in secs:
        i = secs.index(-1)
        secs[i] = n - builtins.sum(s for s in secs if s != -1)
    return [_w(p) for p in torch.split(t, secs, dim=axis)]


def tensor_split(x, num_or_indices, axis=0, name=None):
    return [_w(p) for p in torch.tensor_split(_u(x), num_or_indices, dim=axis)]


def hsplit(x, num_or_indices, name=None):
    return [_w(p) for p in torch.hsplit(_u(x), num_or_indices)]


def vsplit(x, num_or_indices, name=None):
    return [_w(p) for p in torch.vsplit(_u(x), num_or_indices)]


def dsplit(x, num_or_indices, name=None):
    return [_w(p) for p in torch.dsplit(_u(x), num_or_indices)]


def chunk(x, chunks, axis=0, name=None):
    return split(x, chunks, axis)


def unbind(input, axis=0):  # noqa: A002
    return [_w(p) for p in torch.unbind(_u(input), dim=axis)]


def unstack(x, axis=0, num=None):
    return unbind(x, axis)


def squeeze(x, axis=None, name=None):
    t = _u(x)
    a = _axis(axis)
    if a is None:
        return _w(t.squeeze())
    if isinstance(a, int):
        a = (a,)
    dims = tuple(d for d in a if t.shape[d] == 1)
    return _w(t.squeeze(dims) if dims else t)


def squeeze_(x, axis=None, name=None):
    x._t = squeeze(x, axis)._t
    return x


def unsqueeze(x, axis, name=None):
    t = _u(x)
    a = _axis(axis)
    if isinstance(a, int):
        return _w(t.unsqueeze(a))
    for d in a:
        t = t.unsqueeze(d)
    return _w(t)


def unsqueeze_(x, axis, name=None):
    x._t = unsqueeze(x, axis)._t
    return x


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    t = _u(x)
    if t.dim() == 0:
        return _w(t.reshape(1))
    return _w(t.flatten(start_axis, stop_axis))


def flatten_(x, start_axis=0, stop_axis=-1, name=None):
    x._t = flatten(x, start_axis, stop_axis)._t
    return x


def unflatten(x, axis, shape, name=None):
    return _w(_u(x).unflatten(axis, _shape(shape)))


def expand(x, shape, name=None):
    t = _u(x)
    return _w(t.expand(*_shape(shape)))


def expand_as(x, y, name=None):
    return _w(_u(x).expand_as(_u(y)))


def broadcast_to(x, shape, name=None):
    return _w(torch.broadcast_to(_u(x), _shape(shape)))


def broadcast_tensors(input, name=None):  # noqa: A002
    return [_w(p) for p in torch.broadcast_tensors(*[_u(e) for e in input])]


def tile(x, repeat_times, name=None):
    return _w(_u(x).repeat(*_shape(repeat_times)) if len(_shape(repeat_times)) >= _u(x).dim()
              else _u(x).tile(tuple(_shape(repeat_times))))


def repeat_interleave(x, repeats, axis=None, name=None):
    return _w(torch.repeat_interleave(_u(x), _u(repeats) if isinstance(repeats, Tensor) else repeats, dim=axis))


def flip(x, axis, name=None):
    a = _axis(axis)
    return _w(torch.flip(_u(x), (a,) if isinstance(a, int) else a))


reverse = flip


def rot90(x, k=1, axes=[0, 1], name=None):  # noqa: B006
    return _w(torch.rot90(_u(x), k, list(axes)))


def roll(x, shifts, axis=None, name=None):
    return _w(torch.roll(_u(x), _shape(shifts) if not isinstance(shifts, int) else shifts,
                         dims=_axis(axis)))


def gather(x, index, axis=None, name=None):
    t, i = _u(x), _u(index)
    axis = 0 if axis is None else (int(_u(axis)) if isinstance(axis, Tensor) else axis)
    if i.dim() == 0:
        return _w(t.index_select(axis, i.reshape(1)).squeeze(axis))
    return _w(t.index_select(axis, i.reshape(-1)))


def gather_nd(x, index, name=None):
    t, i = _u(x), _u(index)
    k = i.shape[-1]
    idx = tuple(i[..., j] for j in range(k))
    return _w(t[idx])


def index_select(x, index, axis=0, name=None):
    return _w(torch.index_select(_u(x), axis, _u(index).reshape(-1)))


def index_sample(x, index):
    return _w(torch.gather(_u(x), 1, _u(index)))


def take_along_axis(arr, indices, axis, broadcast=True):
    t, i = _u(arr), _u(indices)
    if broadcast and t.dim() == i.dim():
        shp = [builtins.max(a, b) if d != axis % t.dim() else b for d, (a, b) in enumerate(zip(t.shape, i.shape))]
        i = i.expand(shp)
        tshp = list(shp)
        tshp[axis] = t.shape[axis]
        t = t.expand(tshp)
    return _w(torch.gather(t, axis, i))


def put_along_axis(arr, indices, values, axis, reduce='assign', include_self=True, broadcast=True):
    t, i = _u(arr), _u(indices)
    v = _t(values, t)
    if not isinstance(v, torch.Tensor):
        v = torch.full(i.shape, v, dtype=t.dtype, device=t.device)
    v = v.to(t.dtype).expand(i.shape) if v.dim() <= i.dim() else v
    if reduce == 'assign':
        return _w(t.scatter(axis, i, v))
    red = {'add': 'sum', 'mul': 'prod', 'multiply': 'prod', 'mean': 'mean', 'amax': 'amax', 'amin': 'amin'}[reduce]
    return _w(t.scatter_reduce(axis, i, v, red, include_self=include_self))


def put_along_axis_(arr, indices, values, axis, reduce='assign', include_self=True, broadcast=True):
    arr._t.copy_(put_along_axis(arr, indices, values, axis, reduce, include_self, broadcast)._t)
    return arr


@_amp_op('scatter')
def scatter(x, index, updates, overwrite=True, name=None):
    t, i, u = _u(x), _u(index).reshape(-1), _u(updates)
    if overwrite:
        out = t.clone()
        out[i] = u
        return _w(out)
    out = t.clone()
    out[i] = 0
    return _w(out.index_add(0, i, u))


def scatter_(x, index, updates, overwrite=True, name=None):
    with torch.no_grad():
        x._t.copy_(scatter(x, index, updates, overwrite)._t)
    return x


def scatter_nd_add(x, index, updates, name=None):
    t, i, u = _u(x), _u(index), _u(updates)
    k = i.shape[-1]
    flat_i = i.reshape(-1, k)
    tail = t.shape[k:]
    u = u.reshape(-1, *tail)
    strides = torch.tensor([int(np.prod(t.shape[j + 1:k])) for j in range(k)], device=t.device, dtype=torch.int64)
    lin = (flat_i.to(torch.int64) * strides).sum(-1)
    out = t.reshape(-1, *tail).index_add(0, lin, u)
    return _w(out.reshape(t.shape))


def scatter_nd(index, updates, shape, name=None):
    u = _u(updates)
    z = torch.zeros(_shape(shape), dtype=u.dtype, device=u.device)
    return scatter_nd_add(_w(z), index, updates)


def index_add(x, index, axis, value, name=None):
    return _w(torch.index_add(_u(x), axis, _u(index), _u(value)))


def index_add_(x, index, axis, value, name=None):
    x._t.index_add_(axis, _u(index), _u(value))
    return x


def index_put(x, indices, value, accumulate=False, name=None):
    return _w(torch.index_put(_u(x), tuple(_u(i) for i in indices), _t(value, _u(x)), accumulate=accumulate))


def index_put_(x, indices, value, accumulate=False, name=None):
    x._t.index_put_(tuple(_u(i) for i in indices), _t(value, x._t), accumulate=accumulate)
    return x


def index_fill(x, index, axis, value, name=None):
    return _w(torch.index_fill(_u(x), axis, _u(index), _t(value)))


def index_fill_(x, index, axis, value, name=None):
    x._t.index_fill_(axis, _u(index), _t(value))
    return x


def masked_fill(x, mask, value, name=None):
    return _w(torch.masked_fill(_u(x), _u(mask), _t(value)))


def masked_fill_(x, mask, value, name=None):
    x._t.masked_fill_(_u(mask), _t(value))
    return x


def masked_scatter(x, mask, value, name=None):
    return _w(torch.masked_scatter(_u(x), _u(mask), _u(value)))


def masked_scatter_(x, mask, value, name=None):
    x._t.masked_scatter_(_u(mask), _u(value))
    return x


def masked_select(x, mask, name=None):
    return _w(torch.masked_select(_u(x), _u(mask)))


def slice(input, axes, starts, ends):  # noqa: A001,A002
    t = _u(input)
    idx = [builtins.slice(None)] * t.dim()
    starts, ends = _shape(starts), _shape(ends)
    for a, s, e in zip(axes, starts, ends):
        n = t.shape[a]
        s = builtins.max(s + n, 0) if s < 0 else builtins.min(s, n)
        e = builtins.max(e + n, 0) if e < 0 else builtins.min(e, n)
        idx[a] = builtins.slice(s, e)
    return _w(t[tuple(idx)])


def strided_slice(x, axes, starts, ends, strides, name=None):
    t = _u(x)
    idx = [builtins.slice(None)] * t.dim()
    flips = []
    for a, s, e, st in zip(axes, _shape(starts), _shape(ends), _shape(strides)):
        n = t.shape[a]
        if st > 0:
            idx[a] = builtins.slice(s, e, st)
        else:
            s = s + n if s < 0 else builtins.min(s, n - 1)
            e = e + n if e < -n else (e + n if e < 0 else e)
            rng = list(range(s, e, st))
            idx[a] = torch.tensor(rng, dtype=torch.long, device=t.device) if rng else builtins.slice(0, 0)
            flips.append(a)
    out = t
    for a, ix in enumerate(idx):
        if isinstance(ix, torch.Tensor):
            out = out.index_select(a, ix)
        else:
            sl = [builtins.slice(None)] * t.dim()
            sl[a] = ix
            out = out[tuple(sl)]
    return _w(out)


def slice_scatter(x, value, axes, starts, ends, strides, name=None):
    out = _u(x).clone()
    idx = [builtins.slice(None)] * out.dim()
    for a, s, e, st in zip(axes, starts, ends, strides):
        idx[a] = builtins.slice(s, e, st)
    out[tuple(idx)] = _u(value)
    return _w(out)


def select_scatter(x, values, axis, index, name=None):
    return _w(torch.select_scatter(_u(x), _u(values), axis, index))


def diagonal_scatter(x, y, offset=0, axis1=0, axis2=1, name=None):
    return _w(torch.diagonal_scatter(_u(x), _u(y), offset, axis1, axis2))


def crop(x, shape=None, offsets=None, name=None):
    t = _u(x)
    shape = _shape(shape) if shape is not None else list(t.shape)
    offsets = _shape(offsets) if offsets is not None else [0] * t.dim()
    shape = [t.shape[i] - offsets[i] if s == -1 else s for i, s in enumerate(shape)]
    return _w(t[tuple(builtins.slice(o, o + s) for o, s in zip(offsets, shape))])


def unique(x, return_index=False, return_inverse=False, return_counts=False, axis=None, dtype='int64', name=None):
    t = _u(x)
    res = torch.unique(t, sorted=True, return_inverse=True, return_counts=True, dim=axis)
    out, inv, cnt = res
    outs = [_w(out)]
    if return_index:
        flat = t if axis is None else None
        if axis is None:
            flat = t.flatten()
            perm = torch.arange(flat.numel(), device=t.device)
            first = torch.full((out.numel(),), flat.numel(), dtype=torch.long, device=t.device)
            first = first.scatter_reduce(0, inv.flatten(), perm, 'amin')
        else:
            perm = torch.arange(t.shape[axis], device=t.device)
            first = torch.full((out.shape[axis],), t.shape[axis], dtype=torch.long, device=t.device)
            first = first.scatter_reduce(0, inv, perm, 'amin')
        outs.append(_w(first.to(_dtype(dtype))))
    if return_inverse:
        outs.append(_w(inv.to(_dtype(dtype))))
    if return_counts:
        outs.append(_w(cnt.to(_dtype(dtype))))
    return outs[0] if len(outs) == 1 else tuple(outs)


def unique_consecutive(x, return_inverse=False, return_counts=False, axis=None, dtype='int64', name=None):
    out, inv, cnt = torch.unique_consecutive(_u(x), return_inverse=True, return_counts=True, dim=axis)
    outs = [_w(out)]
    if return_inverse:
        outs.append(_w(inv.to(_dtype(dtype))))
    if return_counts:
        outs.append(_w(cnt.to(_dtype(dtype))))
    return outs[0] if len(outs) == 1 else tuple(outs)


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):  # noqa: A002
    t = _u(input)
    size = (index_num + nshards - 1) // nshards
    lo = shard_id * size
    inside = (t >= lo) & (t < lo + size)
    return _w(torch.where(inside, t - lo, torch.full_like(t, ignore_value)))


def atleast_1d(*inputs, name=None):
    r = [_w(torch.atleast_1d(_u(i))) for i in inputs]
    return r[0] if len(r) == 1 else r


def atleast_2d(*inputs, name=None):
    r = [_w(torch.atleast_2d(_u(i))) for i in inputs]
    return r[0] if len(r) == 1 else r


def atleast_3d(*inputs, name=None):
    r = [_w(torch.atleast_3d(_u(i))) for i in inputs]
    return r[0] if len(r) == 1 else r


def unfold(x, axis, size, step, name=None):
    return _w(_u(x).unfold(axis, size, step))


def as_complex(x, name=None):
    return _w(torch.view_as_complex(_u(x).contiguous()))


def as_real(x, name=None):
    return _w(torch.view_as_real(_u(x)))


def tolist(x):
    return _u(x).tolist()


def block_diag(inputs, name=None):
    return _w(torch.block_diag(*[_u(i) for i in inputs]))


def multiplex(inputs, index, name=None):
    ts = torch.stack([_u(i) for i in inputs])
    idx = _u(index).reshape(-1).long()
    return _w(ts[idx, torch.arange(ts.shape[1], device=ts.device)])


def fill_diagonal_(x, value, offset=0, wrap=False, name=None):
    t = x._t
    with torch.no_grad():
        if offset == 0:
            t.fill_diagonal_(value, wrap=wrap)
        else:
            n = builtins.min(t.shape[0], t.shape[1] - offset) if offset > 0 else builtins.min(t.shape[0] + offset, t.shape[1])
            r = torch.arange(n, device=t.device)
            if offset > 0:
                t[r, r + offset] = value
            else:
                t[r - offset, r] = value
    return x


def fill_diagonal_tensor(x, y, offset=0, dim1=0, dim2=1, name=None):
    return _w(torch.diagonal_scatter(_u(x), _u(y), offset, dim1, dim2))


def tensordot(x, y, axes=2, name=None):
    if isinstance(axes, Tensor):
        axes = axes.tolist()
    return _w(torch.tensordot(_u(x), _u(y), dims=axes))


def _runtime_shape(x):
    return _w(torch.tensor(list(x._t.shape), dtype=torch.int32))


def shape(input):  # noqa: A002
    t = _u(input)
    if t.is_meta:
        # static mode: a recorded node producing the run-time extents (dynamic dims included), its
        # record-time value kept for the shape inference of consumers
        from ..static.program import py_node
        out = py_node(_runtime_shape, [input], [torch.empty(t.dim(), dtype=torch.int32, device='meta')])[0]
        out.__dict__['_static_value'] = list(t.shape)
        return out
    return _w(torch.tensor(list(t.shape), dtype=torch.int32))


def resize_(x, shape, fill_zero=False):
    x._t.resize_(_shape(shape))
    return x
