"""Reference-format inference programs: ``.pdmodel`` = a serialized ``ProgramDesc``
(paddle/fluid/framework/framework.proto:264) and ``.pdiparams`` = the save_combine stream of
every persistable variable in sorted-name order (static/proto.py).

Export (``export``): the recorded Program (torch-level op list, static/program.py) is lowered
op by op to the reference's operator set — conv2d, pool2d, batch_norm, matmul_v2,
elementwise_*, scale, layer_norm, softmax, activations, reshape2, transpose2,
flatten_contiguous_range, concat, squeeze2/unsqueeze2, reduce_*, lookup_table_v2, cast, dropout
(inference), feed/fetch — with the reference attribute names
(paddle/phi/api/yaml/op_compat.yaml).  A program that uses anything outside that set raises
``Unsupported`` and the caller keeps this framework's own IR format.

Import (``load``): a ProgramDesc (ours or written by the reference's save_inference_model /
jit.save for the same operator subset) becomes a LoadedProgram whose nodes call the operator
implementations of ``OPS`` on torch tensors, so Executor.run, paddle.inference predictors and
jit.load run it unchanged.  Parameters come from the .pdiparams stream.
"""
import math

import torch
import torch.nn.functional as TF

from . import proto as P
from .program import Ref, Const, Node, SENTINELS

_SENT = set(SENTINELS)


class Unsupported(Exception):
    pass


# ============================================================================ attributes
_AT = {n: i for i, n in enumerate(P.ATTR_TYPES)}


def _set_attr(op, name, v):
    a = op.attrs.add()
    a.name = name
    if isinstance(v, bool):
        a.type, a.b = _AT['BOOLEAN'], v
    elif isinstance(v, int):
        if -2 ** 31 <= v < 2 ** 31:
            a.type, a.i = _AT['INT'], v
        else:
            a.type, a.l = _AT['LONG'], v
    elif isinstance(v, float):
        a.type, a.f = _AT['FLOAT'], v
    elif isinstance(v, str):
        a.type, a.s = _AT['STRING'], v
    elif isinstance(v, (list, tuple)):
        vs = list(v)
        if all(isinstance(x, bool) for x in vs) and vs:
            a.type = _AT['BOOLEANS']
            a.bools.extend(vs)
        elif all(isinstance(x, int) for x in vs):
            a.type = _AT['INTS']
            a.ints.extend(vs)
        elif all(isinstance(x, (int, float)) for x in vs):
            a.type = _AT['FLOATS']
            a.floats.extend([float(x) for x in vs])
        else:
            a.type = _AT['STRINGS']
            a.strings.extend([str(x) for x in vs])
    else:
        raise Unsupported(f"attribute {name}={v!r}")


def _get_attr(a):
    t = P.ATTR_TYPES[a.type]
    return {'INT': lambda: a.i, 'FLOAT': lambda: a.f, 'STRING': lambda: a.s, 'INTS': lambda: list(a.ints),
            'FLOATS': lambda: list(a.floats), 'STRINGS': lambda: list(a.strings), 'BOOLEAN': lambda: a.b,
            'BOOLEANS': lambda: list(a.bools), 'LONG': lambda: a.l, 'LONGS': lambda: list(a.longs),
            'FLOAT64': lambda: a.float64, 'FLOAT64S': lambda: list(a.float64s), 'BLOCK': lambda: a.block_idx,
            'BLOCKS': lambda: list(a.blocks_idx), 'VAR': lambda: a.var_name, 'VARS': lambda: list(a.vars_name),
            'SCALAR': lambda: a.scalar, 'SCALARS': lambda: list(a.scalars)}[t]()


# ============================================================================ operator implementations
def _one(ins, k):
    v = ins.get(k)
    return v[0] if v else None


def _bcast_axis(x, y, axis):
    """Reference elementwise broadcast: y's dims align with x's starting at ``axis``."""
    if axis == -1 or y.dim() == x.dim() or y.dim() == 0:
        return y
    shape = [1] * axis + list(y.shape) + [1] * (x.dim() - axis - y.dim())
    return y.reshape(shape)


def _ew(fn):
    def f(ins, at):
        x, y = _one(ins, 'X'), _one(ins, 'Y')
        return {'Out': [fn(x, _bcast_axis(x, y, at.get('axis', -1)))]}
    return f


def _act(fn):
    return lambda ins, at: {'Out': [fn(_one(ins, 'X'), at)]}


def _pool2d(ins, at):
    x = _one(ins, 'X')
    nhwc = at.get('data_format', 'NCHW') == 'NHWC'
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    k, s, p = at.get('ksize', [1, 1]), at.get('strides', [1, 1]), at.get('paddings', [0, 0])
    if len(p) == 4:
        p = [p[0], p[2]]
    typ = at.get('pooling_type', 'max')
    if at.get('global_pooling', False):
        y = x.amax((2, 3), keepdim=True) if typ == 'max' else x.mean((2, 3), keepdim=True)
    elif at.get('adaptive', False):
        y = TF.adaptive_max_pool2d(x, k) if typ == 'max' else TF.adaptive_avg_pool2d(x, k)
    elif typ == 'max':
        y = TF.max_pool2d(x, k, s, p, ceil_mode=at.get('ceil_mode', False))
    else:
        y = TF.avg_pool2d(x, k, s, p, ceil_mode=at.get('ceil_mode', False),
                          count_include_pad=not at.get('exclusive', True))
    return {'Out': [y.permute(0, 2, 3, 1) if nhwc else y]}


def _conv2d(ins, at):
    x, w = _one(ins, 'Input'), _one(ins, 'Filter')
    nhwc = at.get('data_format', 'NCHW') == 'NHWC'
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    p = at.get('paddings', [0, 0])
    alg = at.get('padding_algorithm', 'EXPLICIT')
    if alg == 'SAME':
        pad = 'same'
    elif alg == 'VALID':
        pad = 0
    elif len(p) == 4:
        if p[0] != p[1] or p[2] != p[3]:
            x = TF.pad(x, (p[2], p[3], p[0], p[1]))
            pad = 0
        else:
            pad = (p[0], p[2])
    else:
        pad = tuple(p)
    y = TF.conv2d(x, w, None, at.get('strides', [1, 1]), pad, at.get('dilations', [1, 1]), at.get('groups', 1))
    return {'Output': [y.permute(0, 2, 3, 1) if nhwc else y]}


def _batch_norm(ins, at):
    x = _one(ins, 'X')
    nhwc = at.get('data_layout', 'NCHW') == 'NHWC'
    xt = x.movedim(-1, 1) if nhwc else x
    y = TF.batch_norm(xt, _one(ins, 'Mean'), _one(ins, 'Variance'), _one(ins, 'Scale'), _one(ins, 'Bias'),
                      False, 0.0, at.get('epsilon', 1e-5))
    return {'Y': [y.movedim(1, -1) if nhwc else y]}


def _layer_norm(ins, at):
    x = _one(ins, 'X')
    ax = at.get('begin_norm_axis', 1)
    ns = list(x.shape[ax:])
    w, b = _one(ins, 'Scale'), _one(ins, 'Bias')
    return {'Y': [TF.layer_norm(x, ns, None if w is None else w.reshape(ns), None if b is None else b.reshape(ns),
                                at.get('epsilon', 1e-5))]}


def _matmul_v2(ins, at):
    from ..ops import matmul as _hm  # bf16 / fp16 GPU operands: the hand-written GEMM
    x, y = _one(ins, 'X'), _one(ins, 'Y')
    if at.get('trans_x', False):
        x = x.transpose(-1, -2) if x.dim() > 1 else x
    if at.get('trans_y', False):
        y = y.transpose(-1, -2) if y.dim() > 1 else y
    return {'Out': [_hm.matmul(x, y)]}


def _matmul_v1(ins, at):
    out = _matmul_v2(ins, {'trans_x': at.get('transpose_X', False), 'trans_y': at.get('transpose_Y', False)})
    a = at.get('alpha', 1.0)
    return {'Out': [out['Out'][0] * a if a != 1.0 else out['Out'][0]]}


def _mul(ins, at):
    x, y = _one(ins, 'X'), _one(ins, 'Y')
    xn = at.get('x_num_col_dims', 1)
    x2 = x.reshape(int(math.prod(x.shape[:xn])), -1)
    out = x2 @ y.reshape(x2.shape[1], -1)
    return {'Out': [out.reshape(*x.shape[:xn], -1)]}


def _reshape2(ins, at):
    x = _one(ins, 'X')
    shape = [x.shape[i] if s == 0 else s for i, s in enumerate(at['shape'])]
    return {'Out': [x.reshape(shape)]}


def _reduce(fn):
    def f(ins, at):
        x = _one(ins, 'X')
        if at.get('reduce_all', False) or not at.get('dim', []):
            y = fn(x, list(range(x.dim())), at.get('keep_dim', False))
        else:
            y = fn(x, [d % x.dim() for d in at['dim']], at.get('keep_dim', False))
        return {'Out': [y]}
    return f


def _gelu(x, at):
    return TF.gelu(x, approximate='tanh' if at.get('approximate', False) else 'none')


def _slice(ins, at):
    x = _one(ins, 'Input')
    idx = [slice(None)] * x.dim()
    for a, s, e in zip(at['axes'], at['starts'], at['ends']):
        idx[a] = slice(s, min(e, x.shape[a]))
    y = x[tuple(idx)]
    dec = at.get('decrease_axis', [])
    if dec:
        y = y.squeeze(tuple(dec)) if len(dec) < y.dim() else y.reshape([])
    return {'Out': [y]}


def _squeeze2(ins, at):
    x = _one(ins, 'X')
    ax = [a % x.dim() for a in at.get('axes', [])]
    return {'Out': [x.squeeze(tuple(ax)) if ax else x.squeeze()]}


def _unsqueeze2(ins, at):
    x = _one(ins, 'X')
    for a in sorted(at.get('axes', [])):
        x = x.unsqueeze(a)
    return {'Out': [x]}


def _cast(ins, at):
    return {'Out': [_one(ins, 'X').to(P.torch_dtype(at['out_dtype']))]}


def _scale(ins, at):
    x = _one(ins, 'X')
    s, b = at.get('scale', 1.0), at.get('bias', 0.0)
    return {'Out': [x * s + b if at.get('bias_after_scale', True) else (x + b) * s]}


def _lookup(ins, at):
    ids, w = _one(ins, 'Ids'), _one(ins, 'W')
    out = TF.embedding(ids.long(), w)
    pi = at.get('padding_idx', -1)
    if pi is not None and pi >= 0:
        out = out * (ids != pi).unsqueeze(-1).to(out.dtype)
    return {'Out': [out]}


def _quant_linear_op(ins, at, quant):
    """quantize_linear / dequantize_linear (reference onnx_format int8 models): abs-max ``Scale``
    (per tensor, or per channel along quant_axis), symmetric (zero point 0).  quantize returns the
    integer grid values (in X's float dtype), dequantize maps them back."""
    x, sc = _one(ins, 'X'), _one(ins, 'Scale')
    qmax = float(2 ** (at.get('bit_length', 8) - 1) - 1)
    axis = at.get('quant_axis', -1)
    s = sc.to(x.device).float()
    if axis is not None and axis >= 0 and s.numel() > 1:
        shape = [1] * x.dim()
        shape[axis] = -1
        s = s.reshape(shape)
    step = s / qmax
    if quant:
        return torch.round(x.float() / step).clamp(-qmax, qmax).to(x.dtype if x.is_floating_point() else torch.float32)
    out = x.float() * step
    return out


def _dropout(ins, at):
    x = _one(ins, 'X')
    p = at.get('dropout_prob', 0.5)
    impl = at.get('dropout_implementation', 'downgrade_in_infer')
    return {'Out': [x * (1.0 - p) if impl == 'downgrade_in_infer' else x]}


# ---- widened set: the operators the reference's jit.save / save_inference_model write for the
# vision zoo (interp, pad, conv transpose, group / instance norm, prelu, fc), ERNIE / GPT
# (fill_constant, shape, stack, gather, where, tril_triu, split, expand_v2, range, comparisons,
# cumsum, top_k_v2, one_hot_v2, index_select) — legacy slot / attribute names of
# paddle/phi/api/yaml/op_compat.yaml.
def _fill_constant(ins, at):
    shape = at.get('shape', [])
    st = ins.get('ShapeTensor') or []
    if st:
        shape = [int(v) for v in st[0].reshape(-1).tolist()]
    val = at.get('value', 0.0)
    if at.get('str_value'):
        val = float(at['str_value'])
    vt = ins.get('ValueTensor') or []
    if vt:
        val = vt[0].reshape(-1)[0].item()
    return {'Out': [torch.full(list(shape), val, dtype=P.torch_dtype(at.get('dtype', 5)))]}


def _stack(ins, at):
    return {'Y': [torch.stack(ins['X'], at.get('axis', 0))]}


def _gather(ins, at):
    x, idx = _one(ins, 'X'), _one(ins, 'Index')
    ax = at.get('axis', 0)
    if ins.get('Axis'):
        ax = int(ins['Axis'][0].reshape(-1)[0])
    return {'Out': [torch.index_select(x, ax, idx.reshape(-1).long()).reshape(
        list(x.shape[:ax]) + list(idx.shape) + list(x.shape[ax + 1:]) if idx.dim() != 1 else
        list(x.shape[:ax]) + [idx.shape[0]] + list(x.shape[ax + 1:]))]}


def _split(ins, at):
    x = _one(ins, 'X')
    ax = at.get('axis', 0)
    if ins.get('AxisTensor'):
        ax = int(ins['AxisTensor'][0].reshape(-1)[0])
    ax %= x.dim()
    sec = at.get('sections', [])
    if sec:
        sec = list(sec)
        if -1 in sec:
            sec[sec.index(-1)] = x.shape[ax] - (sum(sec) + 1)
        return {'Out': list(torch.split(x, sec, ax))}
    return {'Out': list(torch.chunk(x, at.get('num', 1), ax))}


def _expand_v2(ins, at):
    x = _one(ins, 'X')
    shape = list(at.get('shape', []))
    if ins.get('Shape'):
        shape = [int(v) for v in ins['Shape'][0].reshape(-1).tolist()]
    lead = len(shape) - x.dim()
    shape = [x.shape[i - lead] if s == -1 else s for i, s in enumerate(shape)]
    return {'Out': [x.expand(shape)]}


def _cmp(fn):
    return lambda ins, at: {'Out': [fn(_one(ins, 'X'), _one(ins, 'Y'))]}


def _cumsum(ins, at):
    x = _one(ins, 'X')
    if at.get('flatten', False):
        x = x.reshape(-1)
    ax = at.get('axis', -1)
    if at.get('reverse', False):
        x = x.flip(ax)
    y = x.cumsum(ax)
    if at.get('exclusive', False):
        y = y - x
    return {'Out': [y.flip(ax) if at.get('reverse', False) else y]}


def _top_k_v2(ins, at):
    x = _one(ins, 'X')
    k = at.get('k', 1)
    if ins.get('K'):
        k = int(ins['K'][0].reshape(-1)[0])
    v, i = torch.topk(x, k, at.get('axis', -1), largest=at.get('largest', True), sorted=at.get('sorted', True))
    return {'Out': [v], 'Indices': [i]}


def _interp(mode):
    def f(ins, at):
        x = _one(ins, 'X')
        nhwc = at.get('data_layout', 'NCHW') == 'NHWC'
        if nhwc:
            x = x.permute(0, 3, 1, 2)
        oh, ow = at.get('out_h', -1), at.get('out_w', -1)
        if ins.get('OutSize'):
            oh, ow = [int(v) for v in ins['OutSize'][0].reshape(-1).tolist()]
        sc = at.get('scale', [])
        kw = {}
        if oh > 0 and ow > 0:
            kw['size'] = (oh, ow)
        else:
            kw['scale_factor'] = tuple(sc) if len(sc) == 2 else (sc[0], sc[0])
        if mode == 'nearest':
            y = TF.interpolate(x, mode='nearest', **kw)
        else:
            y = TF.interpolate(x, mode=mode, align_corners=at.get('align_corners', False), **kw)
        return {'Out': [y.permute(0, 2, 3, 1) if nhwc else y]}
    return f


def _pad3d(ins, at):
    x = _one(ins, 'X')
    p = at.get('paddings', [0] * 6)  # [left, right, top, bottom, front, back]
    mode = at.get('mode', 'constant')
    ndhwc = at.get('data_format', 'NCDHW') == 'NDHWC'
    if ndhwc:
        x = x.permute(0, 4, 1, 2, 3)
    y = TF.pad(x, list(p), mode=mode, value=at.get('value', 0.0)) if mode == 'constant' else TF.pad(x, list(p), mode=mode)
    return {'Out': [y.permute(0, 2, 3, 4, 1) if ndhwc else y]}


def _conv2d_transpose(ins, at):
    x, w = _one(ins, 'Input'), _one(ins, 'Filter')
    nhwc = at.get('data_format', 'NCHW') == 'NHWC'
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    p = at.get('paddings', [0, 0])
    pad = (p[0], p[2]) if len(p) == 4 else tuple(p)
    op = at.get('output_padding', []) or [0, 0]
    y = TF.conv_transpose2d(x, w, None, at.get('strides', [1, 1]), pad, tuple(op), at.get('groups', 1),
                            at.get('dilations', [1, 1]))
    return {'Output': [y.permute(0, 2, 3, 1) if nhwc else y]}


def _group_norm(ins, at):
    x = _one(ins, 'X')
    nhwc = at.get('data_layout', 'NCHW') == 'NHWC'
    xt = x.movedim(-1, 1) if nhwc else x
    y = TF.group_norm(xt, at.get('groups', 1), _one(ins, 'Scale'), _one(ins, 'Bias'), at.get('epsilon', 1e-5))
    return {'Y': [y.movedim(1, -1) if nhwc else y]}


def _instance_norm(ins, at):
    x = _one(ins, 'X')
    return {'Y': [TF.instance_norm(x, weight=_one(ins, 'Scale'), bias=_one(ins, 'Bias'), eps=at.get('epsilon', 1e-5))]}


def _prelu(ins, at):
    x, a = _one(ins, 'X'), _one(ins, 'Alpha')
    mode = at.get('mode', 'all')
    if mode == 'channel':
        shp = [1, -1] + [1] * (x.dim() - 2) if at.get('data_format', 'NCHW') == 'NCHW' else [1] * (x.dim() - 1) + [-1]
        a = a.reshape(shp)
    elif mode == 'element':
        a = a.reshape([1] + list(x.shape[1:]))
    return {'Out': [torch.where(x >= 0, x, a * x)]}


def _fc(ins, at):
    from ..ops import matmul as _hm
    x, w, b = _one(ins, 'Input'), _one(ins, 'W'), _one(ins, 'Bias')
    n = at.get('in_num_col_dims', 1)
    x2 = x.reshape(int(math.prod(x.shape[:n])), -1)
    y = _hm.matmul(x2, w)
    if b is not None:
        y = y + b.reshape(1, -1)
    if at.get('activation_type', '') == 'relu':
        y = torch.relu(y)
    return {'Out': [y.reshape(*x.shape[:n], -1)]}


def _p_norm(ins, at):
    x = _one(ins, 'X')
    p = at.get('porder', 2.0)
    if at.get('asvector', False):
        return {'Out': [torch.linalg.vector_norm(x.reshape(-1), p)]}
    return {'Out': [torch.linalg.vector_norm(x, p, dim=at.get('axis', -1), keepdim=at.get('keepdim', False))]}


def _assign_value(ins, at):
    dt = P.torch_dtype(at.get('dtype', 5))
    for k in ('fp32_values', 'int32_values', 'int64_values', 'bool_values', 'fp64_values'):
        if at.get(k):
            return {'Out': [torch.tensor(at[k], dtype=dt).reshape(at.get('shape', [-1]))]}
    vals = at.get('values', [])
    return {'Out': [torch.tensor(vals, dtype=dt).reshape(at.get('shape', [-1]))]}


def _fold(x, dims, keep, fn):
    """A one-axis reduction applied over several axes (highest first, so indices stay valid)."""
    for d in sorted(dims, reverse=True):
        x = fn(x, d, keepdim=keep)
    return x


def _arange(ins, at):
    s, e, st = (_one(ins, k).reshape(-1)[0].item() for k in ('Start', 'End', 'Step'))
    return {'Out': [torch.arange(s, e, st, dtype=_one(ins, 'Start').dtype)]}


OPS_EXTRA = {
    'fill_constant': _fill_constant,
    'shape': lambda ins, at: {'Out': [torch.tensor(list(_one(ins, 'Input').shape), dtype=torch.int32)]},
    'stack': _stack, 'gather': _gather,
    'where': lambda ins, at: {'Out': [torch.where(_one(ins, 'Condition').bool(), _one(ins, 'X'), _one(ins, 'Y'))]},
    'tril_triu': lambda ins, at: {'Out': [(torch.tril if at.get('lower', True) else torch.triu)(
        _one(ins, 'X'), at.get('diagonal', 0))]},
    'split': _split, 'expand_v2': _expand_v2,
    'tile': lambda ins, at: {'Out': [_one(ins, 'X').repeat(*(
        [1] * (len(at['repeat_times']) - _one(ins, 'X').dim()) + list(at['repeat_times'])))]},
    'range': _arange,
    'equal': _cmp(torch.eq), 'not_equal': _cmp(torch.ne), 'less_than': _cmp(torch.lt),
    'less_equal': _cmp(torch.le), 'greater_than': _cmp(torch.gt), 'greater_equal': _cmp(torch.ge),
    'logical_and': _cmp(torch.logical_and), 'logical_or': _cmp(torch.logical_or),
    'logical_xor': _cmp(torch.logical_xor),
    'logical_not': lambda ins, at: {'Out': [torch.logical_not(_one(ins, 'X'))]},
    'cumsum': _cumsum, 'top_k_v2': _top_k_v2,
    'one_hot_v2': lambda ins, at: {'Out': [TF.one_hot(_one(ins, 'X').long(), at['depth']).float()]},
    'index_select': lambda ins, at: {'Out': [torch.index_select(_one(ins, 'X'), at.get('dim', 0),
                                                                _one(ins, 'Index').long())]},
    'sin': _act(lambda x, a: torch.sin(x)), 'cos': _act(lambda x, a: torch.cos(x)),
    'log': _act(lambda x, a: torch.log(x)), 'square': _act(lambda x, a: x * x),
    'sign': _act(lambda x, a: torch.sign(x)), 'floor': _act(lambda x, a: torch.floor(x)),
    'ceil': _act(lambda x, a: torch.ceil(x)), 'round': _act(lambda x, a: torch.round(x)),
    'reciprocal': _act(lambda x, a: torch.reciprocal(x)), 'erf': _act(lambda x, a: torch.erf(x)),
    'softplus': _act(lambda x, a: TF.softplus(x, a.get('beta', 1.0), a.get('threshold', 20.0))),
    'mish': _act(lambda x, a: TF.mish(x)), 'elu': _act(lambda x, a: TF.elu(x, a.get('alpha', 1.0))),
    'selu': _act(lambda x, a: TF.selu(x)), 'celu': _act(lambda x, a: TF.celu(x, a.get('alpha', 1.0))),
    'pow': _act(lambda x, a: torch.pow(x, a.get('factor', 1.0))),
    'elementwise_floordiv': _ew(torch.floor_divide), 'elementwise_mod': _ew(torch.remainder),
    'reduce_min': _reduce(lambda x, d, k: x.amin(d, keepdim=k)),
    'reduce_prod': _reduce(lambda x, d, k: _fold(x, d, k, torch.prod)),
    'reduce_any': _reduce(lambda x, d, k: _fold(x.bool(), d, k, torch.any)),
    'reduce_all': _reduce(lambda x, d, k: _fold(x.bool(), d, k, torch.all)),
    'p_norm': _p_norm,
    'bilinear_interp_v2': _interp('bilinear'), 'nearest_interp_v2': _interp('nearest'),
    'bicubic_interp_v2': _interp('bicubic'),
    'pad3d': _pad3d, 'conv2d_transpose': _conv2d_transpose, 'group_norm': _group_norm,
    'instance_norm': _instance_norm, 'prelu': _prelu, 'fc': _fc,
    'argsort': lambda ins, at: dict(zip(('Out', 'Indices'), ([t] for t in torch.sort(
        _one(ins, 'X'), at.get('axis', -1), descending=at.get('descending', False))))),
    'arg_min': lambda ins, at: {'Out': [torch.argmin(_one(ins, 'X'), at.get('axis', -1),
                                                     keepdim=at.get('keepdims', False))]},
    'flip': lambda ins, at: {'Out': [torch.flip(_one(ins, 'X'), list(at.get('axis', [0])))]},
    'roll': lambda ins, at: {'Out': [torch.roll(_one(ins, 'X'), list(at.get('shifts', [0])),
                                                list(at.get('axis', [])) or None)]},
    'unstack': lambda ins, at: {'Y': list(torch.unbind(_one(ins, 'X'), at.get('axis', 0)))},
    'sum': lambda ins, at: {'Out': [sum(ins['X'][1:], ins['X'][0])]},
    'bmm': lambda ins, at: _matmul_v2(ins, {}),
    'fill_any_like': lambda ins, at: {'Out': [torch.full_like(
        _one(ins, 'X'), at.get('value', 0.0), dtype=None if at.get('dtype', -1) in (-1, None) else
        P.torch_dtype(at['dtype']))]},
    'fill_zeros_like': lambda ins, at: {'Out': [torch.zeros_like(_one(ins, 'X'))]},
    'assign_value': _assign_value,
    'lookup_table': _lookup,
    'swish': _act(lambda x, a: x * torch.sigmoid(a.get('beta', 1.0) * x)),
    'hard_sigmoid_': None,
}
OPS_EXTRA.pop('hard_sigmoid_')


OPS = {
    'conv2d': _conv2d, 'depthwise_conv2d': _conv2d, 'pool2d': _pool2d, 'batch_norm': _batch_norm,
    'layer_norm': _layer_norm, 'matmul_v2': _matmul_v2, 'matmul': _matmul_v1, 'mul': _mul,
    'elementwise_add': _ew(torch.add), 'elementwise_sub': _ew(torch.sub), 'elementwise_mul': _ew(torch.mul),
    'elementwise_div': _ew(torch.div), 'elementwise_max': _ew(torch.maximum), 'elementwise_min': _ew(torch.minimum),
    'elementwise_pow': _ew(torch.pow),
    'relu': _act(lambda x, a: torch.relu(x)), 'relu6': _act(lambda x, a: TF.relu6(x)),
    'gelu': _act(_gelu), 'tanh': _act(lambda x, a: torch.tanh(x)), 'sigmoid': _act(lambda x, a: torch.sigmoid(x)),
    'silu': _act(lambda x, a: TF.silu(x)), 'swish': _act(lambda x, a: TF.silu(x)),
    'exp': _act(lambda x, a: torch.exp(x)), 'sqrt': _act(lambda x, a: torch.sqrt(x)),
    'rsqrt': _act(lambda x, a: torch.rsqrt(x)), 'abs': _act(lambda x, a: torch.abs(x)),
    'leaky_relu': _act(lambda x, a: TF.leaky_relu(x, a.get('alpha', 0.02))),
    'hard_swish': _act(lambda x, a: TF.hardswish(x)), 'hard_sigmoid': _act(
        lambda x, a: torch.clamp(x * a.get('slope', 0.2) + a.get('offset', 0.5), 0, 1)),
    'softmax': _act(lambda x, a: torch.softmax(x, a.get('axis', -1))),
    'log_softmax': _act(lambda x, a: torch.log_softmax(x, a.get('axis', -1))),
    'scale': _scale, 'reshape2': _reshape2, 'reshape': _reshape2,
    'transpose2': lambda ins, at: {'Out': [_one(ins, 'X').permute(at['axis'])]},
    'transpose': lambda ins, at: {'Out': [_one(ins, 'X').permute(at['axis'])]},
    'flatten_contiguous_range': lambda ins, at: {'Out': [_one(ins, 'X').flatten(at.get('start_axis', 1),
                                                                                at.get('stop_axis', -1))]},
    'concat': lambda ins, at: {'Out': [torch.cat(ins['X'], at.get('axis', 0))]},
    'squeeze2': _squeeze2, 'unsqueeze2': _unsqueeze2, 'slice': _slice, 'cast': _cast,
    'reduce_mean': _reduce(lambda x, d, k: x.mean(d, keepdim=k)),
    'reduce_sum': _reduce(lambda x, d, k: x.sum(d, keepdim=k)),
    'reduce_max': _reduce(lambda x, d, k: x.amax(d, keepdim=k)),
    'mean': lambda ins, at: {'Out': [_one(ins, 'X').mean()]},
    'lookup_table_v2': _lookup, 'dropout': _dropout,
    'quantize_linear': lambda ins, at: {'Y': [_quant_linear_op(ins, at, True)]},
    'dequantize_linear': lambda ins, at: {'Y': [_quant_linear_op(ins, at, False)]},
    'expand_as_v2': lambda ins, at: {'Out': [_one(ins, 'X').expand_as(_one(ins, 'Y')) if ins.get('Y') else
                                             _one(ins, 'X').expand(at['target_shape'])]},
    'assign': lambda ins, at: {'Out': [_one(ins, 'X')]},
    'clip': lambda ins, at: {'Out': [torch.clamp(_one(ins, 'X'), at.get('min'), at.get('max'))]},
    'arg_max': lambda ins, at: {'Out': [torch.argmax(_one(ins, 'X'), at.get('axis', -1),
                                                     keepdim=at.get('keepdims', False))]},
}
OPS.update(OPS_EXTRA)


# operators whose outputs are made from attributes alone: built on the program's device
_FACTORY_OPS = frozenset({'fill_constant', 'assign_value', 'gaussian_random', 'uniform_random'})


# operators that (re)type values from attributes: under a 16-bit Predictor their fp32 outputs take
# the model dtype (the role of the reference's convert_to_mixed_precision retyping,
# paddle/fluid/inference/analysis/passes/convert_to_mixed_precision.cc)
_RETYPE_OPS = _FACTORY_OPS | {'cast'}


def set_float_dtype(prog, dtype):
    """Make the attribute-typed float values of an imported program (fill_constant, assign_value,
    cast to fp32, ...) ``dtype`` — the whole-program 16-bit mode of the Predictor."""
    for n in prog.nodes:
        if isinstance(n.target, _OpCall) and n.target.type in _RETYPE_OPS:
            n.kwargs = dict(n.kwargs, float_dtype=dtype)
    prog._version = getattr(prog, '_version', 0) + 1


class _OpCall:
    """A node target: runs one reference operator on torch tensors (inputs by slot)."""

    def __init__(self, typ, slots, out_slots, attrs):
        self.type, self.slots, self.out_slots, self.attrs = typ, slots, out_slots, attrs
        self.__name__ = typ

    def __call__(self, *args, device=None, float_dtype=None):
        if device is not None and not any(isinstance(a, torch.Tensor) for a in args):
            # an attribute-only value (fill_constant / assign_value): made once per device and dtype,
            # a constant of every later run (no operator of this runtime writes its inputs in place)
            key = (str(device), float_dtype)
            c = self.__dict__.setdefault('_const', {})
            if key not in c:
                c[key] = self._run(args, device, float_dtype)
            return list(c[key])
        return self._run(args, device, float_dtype)

    def _run(self, args, device, float_dtype):
        dev = next((a.device for a in args if isinstance(a, torch.Tensor) and a.device.type != 'cpu'), None)
        if dev is not None:  # host-made values (shapes, constants of an older export) meet device ones
            args = [a.to(dev, non_blocking=True) if isinstance(a, torch.Tensor) and a.device.type == 'cpu' else a
                    for a in args]
        ins, i = {}, 0
        for slot, n in self.slots:
            ins[slot] = list(args[i:i + n])
            i += n
        outs = OPS[self.type](ins, self.attrs)
        res = []
        for slot, n in self.out_slots:
            vals = outs.get(slot, [])
            res.extend(vals[:n] + [None] * (n - len(vals)))
        if device is not None:
            res = [r.to(device) if isinstance(r, torch.Tensor) else r for r in res]
        if float_dtype is not None:  # 16-bit inference: fp32 constants / casts follow the model dtype
            res = [r.to(float_dtype) if isinstance(r, torch.Tensor) and r.dtype in (torch.float32, torch.float64)
                   else r for r in res]
        return res


# ============================================================================ import
def is_program_desc(data):
    """ProgramDesc bytes (field 1 tag 0x0A) vs this framework's JSON IR (starts with '{')."""
    return bytes(data[:1]) not in (b'{', b'[')


def load(data):
    """ProgramDesc bytes -> LoadedProgram (block 0, inference ops)."""
    from .io import LoadedProgram
    from ..core.tensor import _wrap
    desc = P.ProgramDesc()
    desc.ParseFromString(data)
    blk = desc.blocks[0]
    prog = LoadedProgram()
    vdesc = {v.name: v for v in blk.vars}
    names = {}        # var name -> Ref / Const

    def ref(name):
        if name not in names:
            v = vdesc.get(name)
            if v is not None and v.persistable and v.type.type == P.VAR_TYPES['LOD_TENSOR']:
                cid = len(prog.consts)
                prog.consts[cid] = None  # filled by load_params
                prog._const_names[cid] = name
                names[name] = Const(cid)
            else:
                names[name] = Ref(next(prog._vid))
        return names[name]

    prog._const_names = {}
    feeds, fetch = [], []
    for op in blk.ops:
        at = {a.name: _get_attr(a) for a in op.attrs}
        if op.type == 'feed':
            name = op.outputs[0].arguments[0]
            feeds.append((at.get('col', len(feeds)), name))
            continue
        if op.type == 'fetch':
            fetch.append((at.get('col', len(fetch)), op.inputs[0].arguments[0]))
            continue
        if op.type not in OPS:
            raise NotImplementedError(f"ProgramDesc operator '{op.type}' is not supported by this runtime")
        slots = [(v.parameter, len(v.arguments)) for v in op.inputs]
        args = [ref(a) for v in op.inputs for a in v.arguments]
        out_slots = [(v.parameter, len(v.arguments)) for v in op.outputs]
        outs = [ref(a).vid if isinstance(ref(a), Ref) else None for v in op.outputs for a in v.arguments]
        if op.type in _FACTORY_OPS:  # created on the executor's device (static/executor.py 'factory')
            prog.nodes.append(Node('torch', _OpCall(op.type, slots, out_slots, at), args, {'device': None}, outs,
                                   {'factory': True}))
        else:
            prog.nodes.append(Node('torch', _OpCall(op.type, slots, out_slots, at), args, {}, outs))
    for _, name in sorted(feeds):
        v = vdesc[name]
        td = v.type.lod_tensor.tensor
        shape = [int(d) for d in td.dims]
        dt = P.torch_dtype(td.data_type)
        vid = ref(name).vid
        prog.feeds[name] = (vid, shape, dt)
        m = torch.empty([max(s, 1) for s in shape], dtype=dt, device='meta')
        prog._val[id(m)] = vid
        prog._keep.append(m)
        var = _wrap(m)
        var._name = name
        prog.named_vars[name] = var
    prog._fetch = [ref(n).vid for _, n in sorted(fetch)]
    prog._fetch_vars = []
    for vid in prog._fetch:
        m = torch.empty(0, device='meta')
        prog._val[id(m)] = vid
        prog._keep.append(m)
        prog._fetch_vars.append(_wrap(m))
    prog._pdmodel = True
    return prog


def load_params(prog, data, device):
    from ..core.tensor import Parameter
    tensors = P.load_combine(data, list(prog._const_names.values()))
    prog._const_owner = {}
    for cid, name in prog._const_names.items():
        t = tensors[name].to(device)
        p = Parameter(t, trainable=t.is_floating_point(), name=name)
        prog.consts[cid] = p._t
        prog._const_owner[cid] = p
    for cid, t in list(prog.consts.items()):  # literal constants of the program (PIR full ops)
        if cid not in prog._const_names and isinstance(t, torch.Tensor):
            prog.consts[cid] = t.to(device)


# ============================================================================ export
class _Exporter:
    def __init__(self, prog):
        self.prog = prog
        self.desc = P.ProgramDesc()
        self.blk = self.desc.blocks.add()
        self.blk.idx, self.blk.parent_idx = 0, -1
        self.desc.version.version = 0
        self.meta = {vid: m for m in prog._keep for vid in [prog._val.get(id(m))] if vid is not None}
        self.vars = {}
        self.params = {}  # name -> tensor
        self.cname = {}
        self.tmp = 0

    # ---- variables
    def _var(self, name, dt=None, shape=None, persistable=False):
        if name in self.vars:
            return name
        v = self.blk.vars.add()
        v.name = name
        v.type.type = P.VAR_TYPES['LOD_TENSOR']
        td = v.type.lod_tensor.tensor
        td.data_type = P.dtype_code(dt) if dt is not None else P.VAR_TYPES['FP32']
        td.dims.extend([int(s) for s in (shape or [])])
        v.persistable = persistable
        self.vars[name] = v
        return name

    def _special(self, name, typ):
        v = self.blk.vars.add()
        v.name = name
        v.type.type = P.VAR_TYPES[typ]
        v.persistable = True
        self.vars[name] = v

    def name_of(self, a):
        if isinstance(a, Ref):
            m = self.meta.get(a.vid)
            shape = [-1 if s in _SENT else s for s in m.shape] if m is not None else []
            return self._var(f"tmp_{a.vid}", m.dtype if m is not None else None, shape)
        if isinstance(a, Const):
            if a.cid not in self.cname:
                owner = getattr(self.prog, '_const_owner', {}).get(a.cid)
                t = self.prog.consts[a.cid]
                nm = owner.name if owner is not None and getattr(owner, 'name', None) else f"const_{a.cid}"
                while nm in self.params and self.params[nm] is not t:
                    nm += '_'
                self.cname[a.cid] = nm
                self.params[nm] = t
                self._var(nm, t.dtype, list(t.shape), persistable=True)
            return self.cname[a.cid]
        raise Unsupported(f"operand {a!r}")

    def rank(self, a):
        if isinstance(a, Ref):
            m = self.meta.get(a.vid)
            if m is None:
                raise Unsupported("unknown rank")
            return m.dim()
        return self.prog.consts[a.cid].dim()

    def new_tmp(self, like=None):
        self.tmp += 1
        return self._var(f"tmp_x{self.tmp}", None if like is None else None, [])

    def op(self, typ, inputs, outputs, **attrs):
        o = self.blk.ops.add()
        o.type = typ
        for k, vs in inputs.items():
            v = o.inputs.add()
            v.parameter = k
            v.arguments.extend(vs if isinstance(vs, list) else [vs])
        for k, vs in outputs.items():
            v = o.outputs.add()
            v.parameter = k
            v.arguments.extend(vs if isinstance(vs, list) else [vs])
        for k, val in attrs.items():
            _set_attr(o, k, val)
        return o


def _lit_int(v):
    if isinstance(v, int) and not isinstance(v, bool):
        return -1 if any(v % s == 0 and v != 0 for s in _SENT) else v
    raise Unsupported(f"non-literal int {v!r}")


def _ints(v):
    if isinstance(v, int):
        return [_lit_int(v)]
    return [_lit_int(x) for x in v]


def _pair(v):
    return list(v) * 2 if isinstance(v, (list, tuple)) and len(v) == 1 else (list(v) if isinstance(v, (list, tuple))
                                                                              else [v, v])


def _emit_opcall(ex, n):
    """An imported operator node re-emitted as the operator it came from."""
    t = n.target
    o = ex.blk.ops.add()
    o.type = t.type
    pos = 0
    for slot, cnt in t.slots:
        v = o.inputs.add()
        v.parameter = slot
        v.arguments.extend([ex.name_of(a) for a in n.args[pos:pos + cnt]])
        pos += cnt
    outs = n.outs if isinstance(n.outs, (list, tuple)) else [n.outs]
    pos = 0
    for slot, cnt in t.out_slots:
        v = o.outputs.add()
        v.parameter = slot
        v.arguments.extend([ex.name_of(Ref(vid)) if vid is not None else ex.new_tmp() for vid in outs[pos:pos + cnt]])
        pos += cnt
    for k, val in t.attrs.items():
        if val is None:
            continue
        _set_attr(o, k, val)


def _emit_quant_linear(ex, n):
    """A frozen int8 GEMM (paddle.ops.int8.quant_linear) as the reference's onnx-format ops:
    quantize_linear -> dequantize_linear on the activation (per-tensor threshold), the int8 weight
    ([N, K] stored, dequantize_linear along quant_axis 0) consumed by matmul_v2(trans_y), + bias."""
    x, qw, ws, acs = n.args[0], n.args[1], n.args[2], n.args[3]
    bias = n.args[4] if len(n.args) > 4 else None
    bits = n.kwargs.get('bits', 8)
    wbits = n.kwargs.get('weight_bits', 8)
    out = ex.name_of(Ref(n.outs))
    zp_a, zp_w = ex.new_tmp(), ex.new_tmp()
    ex.op('fill_constant', {}, {'Out': zp_a}, shape=[1], value=0.0, dtype=P.dtype_code(torch.float32))
    ex.op('fill_constant', {}, {'Out': zp_w}, shape=[1], value=0.0, dtype=P.dtype_code(torch.float32))
    xq, xd, wd = ex.new_tmp(), ex.new_tmp(), ex.new_tmp()
    ex.op('quantize_linear', {'X': ex.name_of(x), 'Scale': ex.name_of(acs), 'ZeroPoint': zp_a}, {'Y': xq},
          bit_length=bits, quant_axis=-1)
    ex.op('dequantize_linear', {'X': xq, 'Scale': ex.name_of(acs), 'ZeroPoint': zp_a}, {'Y': xd},
          bit_length=bits, quant_axis=-1)
    ex.op('dequantize_linear', {'X': ex.name_of(qw), 'Scale': ex.name_of(ws), 'ZeroPoint': zp_w}, {'Y': wd},
          bit_length=wbits, quant_axis=0)
    dst = out if bias is None else ex.new_tmp()
    ex.op('matmul_v2', {'X': xd, 'Y': wd}, {'Out': dst}, trans_x=False, trans_y=True)
    if bias is not None:
        ex.op('elementwise_add', {'X': dst, 'Y': ex.name_of(bias)}, {'Out': out}, axis=-1)


def _emit(ex, n):
    if type(n.target).__name__ == '_OpCall':
        return _emit_opcall(ex, n)
    t = getattr(n.target, '__name__', str(n.target))
    if t == 'quant_linear' and getattr(n.target, '__module__', '').endswith('ops.int8'):
        return _emit_quant_linear(ex, n)
    a, k = list(n.args), dict(n.kwargs)
    out = ex.name_of(Ref(n.outs)) if isinstance(n.outs, int) else None

    def X(i=0):
        return ex.name_of(a[i])

    def scalar(v):
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    if t in ('conv2d',):
        x, w = X(0), ex.name_of(a[1])
        b = a[2] if len(a) > 2 else k.get('bias')
        stride = _pair(a[3] if len(a) > 3 else k.get('stride', 1))
        pad = a[4] if len(a) > 4 else k.get('padding', 0)
        if isinstance(pad, str):
            raise Unsupported("string padding")
        dil = _pair(a[5] if len(a) > 5 else k.get('dilation', 1))
        groups = a[6] if len(a) > 6 else k.get('groups', 1)
        dst = out if b is None else ex.new_tmp()
        ex.op('conv2d', {'Input': x, 'Filter': w}, {'Output': dst}, strides=stride, paddings=_pair(pad),
              dilations=dil, groups=groups, data_format='NCHW', padding_algorithm='EXPLICIT')
        if b is not None:
            ex.op('elementwise_add', {'X': dst, 'Y': ex.name_of(b)}, {'Out': out}, axis=1)
    elif t in ('relu', 'tanh', 'sigmoid', 'silu', 'exp', 'sqrt', 'rsqrt', 'abs', 'relu6', 'hardswish'):
        typ = {'hardswish': 'hard_swish'}.get(t, t)
        ex.op(typ, {'X': X()}, {'Out': out})
    elif t == 'gelu':
        ex.op('gelu', {'X': X()}, {'Out': out}, approximate=k.get('approximate', 'none') == 'tanh')
    elif t in ('softmax', 'log_softmax'):
        dim = a[1] if len(a) > 1 else k.get('dim', -1)
        ex.op(t, {'X': X()}, {'Out': out}, axis=int(dim))
    elif t in ('max_pool2d', 'avg_pool2d'):
        ks = _pair(a[1] if len(a) > 1 else k['kernel_size'])
        st = a[2] if len(a) > 2 else k.get('stride')
        st = ks if st in (None, [], ()) else _pair(st)
        pad = _pair(a[3] if len(a) > 3 else k.get('padding', 0))
        if t == 'max_pool2d':
            if (a[4] if len(a) > 4 else k.get('dilation', 1)) not in (1, (1, 1), [1, 1]) or \
                    k.get('return_indices', False):
                raise Unsupported("max_pool2d dilation / indices")
            ceil = a[5] if len(a) > 5 else k.get('ceil_mode', False)
            ex.op('pool2d', {'X': X()}, {'Out': out}, pooling_type='max', ksize=ks, strides=st, paddings=pad,
                  global_pooling=False, adaptive=False, exclusive=True, ceil_mode=bool(ceil), data_format='NCHW',
                  padding_algorithm='EXPLICIT')
        else:
            ceil = a[4] if len(a) > 4 else k.get('ceil_mode', False)
            cip = a[5] if len(a) > 5 else k.get('count_include_pad', True)
            if (a[6] if len(a) > 6 else k.get('divisor_override')) is not None:
                raise Unsupported("divisor_override")
            ex.op('pool2d', {'X': X()}, {'Out': out}, pooling_type='avg', ksize=ks, strides=st, paddings=pad,
                  global_pooling=False, adaptive=False, exclusive=not cip, ceil_mode=bool(ceil), data_format='NCHW',
                  padding_algorithm='EXPLICIT')
    elif t in ('adaptive_avg_pool2d', 'adaptive_max_pool2d'):
        ex.op('pool2d', {'X': X()}, {'Out': out}, pooling_type='avg' if 'avg' in t else 'max',
              ksize=_pair(a[1] if len(a) > 1 else k['output_size']), strides=[1, 1], paddings=[0, 0],
              global_pooling=False, adaptive=True, exclusive=True, ceil_mode=False, data_format='NCHW',
              padding_algorithm='EXPLICIT')
    elif t == 'batch_norm':
        training = a[5] if len(a) > 5 else k.get('training', False)
        if training:
            raise Unsupported("training batch_norm")
        w = a[3] if len(a) > 3 else k.get('weight')
        b = a[4] if len(a) > 4 else k.get('bias')
        eps = a[7] if len(a) > 7 else k.get('eps', 1e-5)
        if w is None or b is None:
            raise Unsupported("batch_norm without affine")
        extra = [ex.new_tmp() for _ in range(4)]
        ex.op('batch_norm', {'X': X(), 'Scale': ex.name_of(w), 'Bias': ex.name_of(b), 'Mean': ex.name_of(a[1]),
                             'Variance': ex.name_of(a[2])},
              {'Y': out, 'MeanOut': extra[0], 'VarianceOut': extra[1], 'SavedMean': extra[2],
               'SavedVariance': extra[3]}, epsilon=float(eps), momentum=0.9, is_test=True, data_layout='NCHW',
              use_global_stats=True, trainable_statistics=False)
    elif t == 'flatten':
        r = ex.rank(a[0])
        s = a[1] if len(a) > 1 else k.get('start_dim', 0)
        e = a[2] if len(a) > 2 else k.get('end_dim', -1)
        ex.op('flatten_contiguous_range', {'X': X()}, {'Out': out, 'XShape': ex.new_tmp()}, start_axis=s % max(r, 1),
              stop_axis=e % max(r, 1))
    elif t in ('addmm',):
        if len(a) != 3 or k:
            raise Unsupported("addmm with alpha/beta")
        tmp = ex.new_tmp()
        ex.op('matmul_v2', {'X': ex.name_of(a[1]), 'Y': ex.name_of(a[2])}, {'Out': tmp}, trans_x=False, trans_y=False)
        ex.op('elementwise_add', {'X': tmp, 'Y': ex.name_of(a[0])}, {'Out': out}, axis=-1)
    elif t in ('mm', 'matmul', 'bmm'):
        ex.op('matmul_v2', {'X': X(0), 'Y': ex.name_of(a[1])}, {'Out': out}, trans_x=False, trans_y=False)
    elif t == 'linear':
        b = a[2] if len(a) > 2 else k.get('bias')
        dst = out if b is None else ex.new_tmp()
        ex.op('matmul_v2', {'X': X(0), 'Y': ex.name_of(a[1])}, {'Out': dst}, trans_x=False, trans_y=True)
        if b is not None:
            ex.op('elementwise_add', {'X': dst, 'Y': ex.name_of(b)}, {'Out': out}, axis=-1)
    elif t == 'layer_norm':
        ns = a[1] if len(a) > 1 else k['normalized_shape']
        w = a[2] if len(a) > 2 else k.get('weight')
        b = a[3] if len(a) > 3 else k.get('bias')
        eps = a[4] if len(a) > 4 else k.get('eps', 1e-5)
        ins = {'X': X()}
        if w is not None:
            ins['Scale'] = ex.name_of(w)
        if b is not None:
            ins['Bias'] = ex.name_of(b)
        if (w is not None and ex.rank(w) != 1) or len(ns) != 1 and (w is not None):
            raise Unsupported("multi-dim layer_norm weight")
        ex.op('layer_norm', ins, {'Y': out, 'Mean': ex.new_tmp(), 'Variance': ex.new_tmp()},
              begin_norm_axis=ex.rank(a[0]) - len(ns), epsilon=float(eps))
    elif t in ('add', 'sub', 'mul', 'div', '__add__', '__sub__', '__mul__', '__truediv__', '__radd__', '__rmul__',
               'add_', 'mul_', 'true_divide', 'multiply', 'subtract'):
        base = {'__add__': 'add', '__radd__': 'add', '__sub__': 'sub', '__mul__': 'mul', '__rmul__': 'mul',
                '__truediv__': 'div', 'true_divide': 'div', 'multiply': 'mul', 'subtract': 'sub'}.get(t, t.rstrip('_'))
        x, y = a[0], a[1] if len(a) > 1 else k.get('other')
        if k.get('alpha', 1) != 1:
            raise Unsupported("add alpha")
        if scalar(x) and not scalar(y) and base in ('add', 'mul'):
            x, y = y, x
        if scalar(y):
            if base == 'div' and float(y) == 0.0:
                raise Unsupported("division by a zero scalar")
            s, bb = {'add': (1.0, float(y)), 'sub': (1.0, -float(y)), 'mul': (float(y), 0.0),
                     'div': (1.0 / float(y) if base == 'div' else 0.0, 0.0)}[base]
            ex.op('scale', {'X': ex.name_of(x)}, {'Out': out}, scale=s, bias=bb, bias_after_scale=True)
        elif scalar(x):
            raise Unsupported("scalar-first sub/div")
        else:
            ex.op('elementwise_' + base, {'X': ex.name_of(x), 'Y': ex.name_of(y)}, {'Out': out}, axis=-1)
    elif t in ('reshape', 'view'):
        shape = list(a[1:] if len(a) > 2 else a[1])
        xm = ex.meta.get(a[0].vid) if isinstance(a[0], Ref) else None
        tgt = []
        for i, v in enumerate(shape):
            # a dynamic (sentinel) extent kept in place is reshape2's 0 ("copy input dim i"), so at
            # most one -1 is left to infer
            if xm is not None and i < xm.dim() and isinstance(v, int) and v == xm.shape[i] and v in _SENT:
                tgt.append(0)
            else:
                tgt.append(_lit_int(v))
        ex.op('reshape2', {'X': X()}, {'Out': out, 'XShape': ex.new_tmp()}, shape=tgt)
    elif t == 'permute':
        dims = a[1:] if len(a) > 2 else a[1]
        ex.op('transpose2', {'X': X()}, {'Out': out, 'XShape': ex.new_tmp()}, axis=[int(d) for d in dims])
    elif t in ('transpose', 'swapaxes'):
        r = ex.rank(a[0])
        perm = list(range(r))
        d0, d1 = a[1] % r, a[2] % r
        perm[d0], perm[d1] = perm[d1], perm[d0]
        ex.op('transpose2', {'X': X()}, {'Out': out, 'XShape': ex.new_tmp()}, axis=perm)
    elif t == 'cat':
        ts = a[0]
        dim = a[1] if len(a) > 1 else k.get('dim', 0)
        ex.op('concat', {'X': [ex.name_of(x) for x in ts]}, {'Out': out}, axis=int(dim))
    elif t in ('unsqueeze', 'squeeze'):
        dim = a[1] if len(a) > 1 else k.get('dim')
        dims = [] if dim is None else ([dim] if isinstance(dim, int) else list(dim))
        ex.op(t + '2', {'X': X()}, {'Out': out, 'XShape': ex.new_tmp()}, axes=dims)
    elif t in ('mean', 'sum') and len(a) >= 1:
        dim = a[1] if len(a) > 1 else k.get('dim')
        keep = a[2] if len(a) > 2 else k.get('keepdim', False)
        if k.get('dtype') is not None:
            raise Unsupported("reduce dtype")
        dims = [] if dim is None else ([dim] if isinstance(dim, int) else list(dim))
        ex.op('reduce_' + t, {'X': X()}, {'Out': out}, dim=dims, keep_dim=bool(keep), reduce_all=not dims)
    elif t == 'embedding':
        pi = k.get('padding_idx', a[2] if len(a) > 2 else None)
        ex.op('lookup_table_v2', {'Ids': X(0), 'W': ex.name_of(a[1])}, {'Out': out},
              padding_idx=-1 if pi is None else int(pi))
    elif t in ('dropout', 'contiguous', 'clone', 'detach'):
        if t == 'dropout' and (a[2] if len(a) > 2 else k.get('training', True)):
            raise Unsupported("training dropout")
        ex.op('assign', {'X': X()}, {'Out': out})
    elif t in ('to', 'float', 'half', 'bfloat16', 'type'):
        dt = {'float': torch.float32, 'half': torch.float16, 'bfloat16': torch.bfloat16}.get(t)
        if dt is None:
            dt = next((v for v in list(a[1:]) + list(k.values()) if isinstance(v, torch.dtype)), None)
        if dt is None:
            raise Unsupported("to() without dtype")
        ex.op('cast', {'X': X()}, {'Out': out}, in_dtype=P.dtype_code(ex.meta[a[0].vid].dtype)
              if isinstance(a[0], Ref) and a[0].vid in ex.meta else 5, out_dtype=P.dtype_code(dt))
    elif t in ('ne', 'eq', 'lt', 'le', 'gt', 'ge', '__ne__', '__eq__', '__lt__', '__le__', '__gt__', '__ge__') \
            and len(a) == 2:
        typ = {'ne': 'not_equal', 'eq': 'equal', 'lt': 'less_than', 'le': 'less_equal', 'gt': 'greater_than',
               'ge': 'greater_equal'}[t.strip('_')]
        y = a[1]
        if scalar(y):
            c = ex.new_tmp()
            xm = ex.meta.get(a[0].vid) if isinstance(a[0], Ref) else None
            ex.op('fill_constant', {}, {'Out': c}, shape=[1], value=float(y),
                  dtype=P.dtype_code(xm.dtype if xm is not None else torch.float32))
            yname = c
        else:
            yname = ex.name_of(y)
        ex.op(typ, {'X': X(), 'Y': yname}, {'Out': out}, axis=-1)
    elif t == 'arange' and len(a) == 1 and scalar(a[0]):
        n_ = _lit_int(a[0])
        if n_ < 0:
            raise Unsupported("arange over a dynamic dim")
        ex.op('assign_value', {}, {'Out': out}, shape=[n_], dtype=P.dtype_code(torch.int64),
              int64_values=list(range(n_)))
    elif t == 'expand_as':
        ex.op('expand_as_v2', {'X': X(), 'Y': ex.name_of(a[1])}, {'Out': out})
    elif t in ('zeros_like', 'ones_like'):
        dt = k.get('dtype') or (ex.meta[a[0].vid].dtype if isinstance(a[0], Ref) and a[0].vid in ex.meta else None)
        ex.op('fill_any_like', {'X': X()}, {'Out': out}, value=0.0 if t == 'zeros_like' else 1.0,
              dtype=P.dtype_code(dt) if dt is not None else -1)
    elif t == 'bool':
        ex.op('cast', {'X': X()}, {'Out': out}, in_dtype=P.dtype_code(ex.meta[a[0].vid].dtype)
              if isinstance(a[0], Ref) and a[0].vid in ex.meta else 3, out_dtype=P.dtype_code(torch.bool))
    elif t in ('__invert__', 'logical_not', 'bitwise_not'):
        xm = ex.meta.get(a[0].vid) if isinstance(a[0], Ref) else None
        if xm is not None and xm.dtype != torch.bool:
            raise Unsupported("bitwise not of a non-bool tensor")
        ex.op('logical_not', {'X': X()}, {'Out': out})
    elif t == 'masked_fill' and len(a) == 3 and scalar(a[2]):
        c = ex.new_tmp()
        xm = ex.meta.get(a[0].vid) if isinstance(a[0], Ref) else None
        ex.op('fill_constant', {}, {'Out': c}, shape=[1], value=float(a[2]),
              dtype=P.dtype_code(xm.dtype if xm is not None else torch.float32))
        ex.op('where', {'Condition': ex.name_of(a[1]), 'X': c, 'Y': X()}, {'Out': out})
    elif t == '__getitem__':
        key = a[1] if isinstance(a[1], tuple) else (a[1],)
        axes, starts, ends, dec = [], [], [], []
        for ax, kk in enumerate(key):
            if isinstance(kk, slice):
                if kk.step not in (None, 1):
                    raise Unsupported("strided slice")
                if kk.start is None and kk.stop is None:
                    continue
                axes.append(ax)
                starts.append(_lit_int(kk.start or 0))
                ends.append(_lit_int(kk.stop) if kk.stop is not None else 2 ** 31 - 1)
            elif isinstance(kk, int) and not isinstance(kk, bool) and kk >= 0:
                axes.append(ax)
                starts.append(kk)
                ends.append(kk + 1)
                dec.append(ax)
            else:
                raise Unsupported(f"index {kk!r}")
        if not axes:
            ex.op('assign', {'X': X()}, {'Out': out})
        else:
            ex.op('slice', {'Input': X()}, {'Out': out}, axes=axes, starts=starts, ends=ends, decrease_axis=dec,
                  infer_flags=[1] * len(axes))
    elif t in ('clamp', 'clip'):
        lo = a[1] if len(a) > 1 else k.get('min')
        hi = a[2] if len(a) > 2 else k.get('max')
        if not all(v is None or scalar(v) for v in (lo, hi)):
            raise Unsupported("tensor clip bounds")
        ex.op('clip', {'X': X()}, {'Out': out}, min=float(-3.4e38 if lo is None else lo),
              max=float(3.4e38 if hi is None else hi))
    else:
        raise Unsupported(f"op '{t}'")


def export(prog, feed_names, fetch_vids):
    """Recorded Program -> (ProgramDesc bytes, [(param name, tensor)])."""
    ex = _Exporter(prog)
    ex._special('feed', 'FEED_MINIBATCH')
    ex._special('fetch', 'FETCH_LIST')
    for i, name in enumerate(feed_names):
        vid, shape, dt = prog.feeds[name]
        ex._var(name, dt, [int(s) for s in shape])
        ex.vars[name].need_check_feed = True
        ex.op('feed', {'X': 'feed'}, {'Out': name}, col=i)
    feed_vid = {prog.feeds[n][0]: n for n in feed_names}
    ex.meta.update({})
    # feed values keep their names
    orig = ex.name_of

    def name_of(a):
        if isinstance(a, Ref) and a.vid in feed_vid:
            return feed_vid[a.vid]
        return orig(a)
    ex.name_of = name_of
    for n in prog.nodes:
        if n.kind != 'torch':
            raise Unsupported(f"node kind {n.kind}")
        if not isinstance(n.outs, int) and type(n.target).__name__ != '_OpCall':
            raise Unsupported("multi-output node")
        _emit(ex, n)
    for i, vid in enumerate(fetch_vids):
        ex.op('fetch', {'X': ex.name_of(Ref(vid))}, {'Out': 'fetch'}, col=i)
    return ex.desc.SerializeToString(), sorted(ex.params.items())
