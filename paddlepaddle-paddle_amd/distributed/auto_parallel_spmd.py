"""Semi-auto parallel SPMD propagation for dygraph dist tensors.

Reference: the per-op SPMD rules of paddle/phi/infermeta/spmd_rules/ (einsum-notation sharding
merge — matmul.cc:117 MatmulInferSpmd, elementwise.cc:231, reduction.cc:68, softmax.cc:30,
layer_norm.cc:49, embedding.cc:31 (vocab-parallel unsupported variant), transpose.cc:50,
reshape.cc:153) and the dygraph dist-op flow: InferSpmd -> reshard the inputs -> run the local
kernel -> set the output's dist attr.

Design here: a dist tensor is a torch tensor holding this rank's local piece, tagged with
``_pd_dist = (mesh, placements, global_shape)``.  While any dist tensor exists, a
``TorchFunctionMode`` sees every torch op; ops with a rule and at least one tagged input run

    rule(shapes, dims_mappings) -> required input dims_mappings, output dims_mapping, partial dims
    inputs  -> differentiable reshards (all-gather / slice / all-reduce / reduce-scatter / all-to-all)
    local op on the local pieces
    output  -> tagged with the inferred placements (Partial on contracted mesh dims)

Gradients are exact by construction: every reshard is an autograd Function whose backward is the
conjugate collective (all-gather <-> slice, all-reduce <-> identity, reduce-scatter <-> all-gather),
and an input that is *replicated* along a mesh dim on which the op's output is sharded or partial
gets an identity-forward / all-reduce-backward marker (its local gradient is a partial sum there).
That yields tensor parallelism (column/row-parallel matmuls) and data parallelism (replicated
weights, batch-sharded activations: the weight gradient is all-reduced) from placements alone.
Ops without a rule run on the local pieces unchanged (the pre-existing local semantics).
"""
import contextlib
import math

import torch
import torch.distributed as dist
from torch.overrides import TorchFunctionMode

_ALPHA = 'abcdefghijklmnopqrstuvwxyz'


# ------------------------------------------------------------------ metadata
def meta(t):
    return getattr(t, '_pd_dist', None) if isinstance(t, torch.Tensor) else None


def tag(t, mesh, placements, gshape):
    t._pd_dist = (mesh, list(placements), list(gshape))
    return t


def _ap():
    from . import auto_parallel as ap
    return ap


def dims_mapping(placements, ndim):
    ap = _ap()
    dm = [-1] * ndim
    for d, p in enumerate(placements):
        if isinstance(p, ap.Shard) and ndim > 0:
            k = p.dim % ndim
            if dm[k] == -1:
                dm[k] = d
    return dm


def partial_dims(placements):
    ap = _ap()
    return {d: p.reduce_type for d, p in enumerate(placements) if isinstance(p, ap.Partial)}


def placements_of(dm, partial, mesh_ndim):
    ap = _ap()
    pl = [ap.Replicate() for _ in range(mesh_ndim)]
    for t, d in enumerate(dm):
        if d >= 0:
            pl[d] = ap.Shard(t)
    for d, rt in partial.items():
        pl[d] = ap.Partial(rt)
    return pl


# ------------------------------------------------------------------ einsum sharding merge
def merge(axes_list, dms):
    """axis letter -> mesh dim; first tensor wins, a mesh dim shards at most one axis."""
    amap, used = {}, set()
    for axes, dm in zip(axes_list, dms):
        for a, d in zip(axes, dm):
            if d < 0 or a == '1' or a in amap or d in used:
                continue
            amap[a] = d
            used.add(d)
    return amap


def einsum_rule(in_axes, in_dms, out_axes, replicate_axes=()):
    amap = merge(in_axes, in_dms)
    for a in replicate_axes:
        amap.pop(a, None)
    req = [[amap.get(a, -1) if a != '1' else -1 for a in axes] for axes in in_axes]
    out = [amap.get(a, -1) if a != '1' else -1 for a in out_axes]
    partial = {d for a, d in amap.items() if a not in out_axes}
    return req, out, partial


def _bcast_axes(shapes):
    n = max(len(s) for s in shapes)
    out_shape = [1] * n
    for s in shapes:
        for i, v in enumerate(s):
            j = n - len(s) + i
            out_shape[j] = max(out_shape[j], v)
    letters = _ALPHA[:n]
    axes = []
    for s in shapes:
        ax = ''
        for i, v in enumerate(s):
            j = n - len(s) + i
            ax += '1' if (v == 1 and out_shape[j] != 1) else letters[j]
        axes.append(ax)
    return axes, letters


def rule_elementwise(shapes, dms):
    axes, out = _bcast_axes(shapes)
    return einsum_rule(axes, dms, out)


def rule_matmul(shapes, dms, trans_x=False, trans_y=False):
    xs, ys = shapes
    xd, yd = list(dms[0]), list(dms[1])
    xn, yn = len(xs), len(ys)
    if trans_x and xn >= 2:
        xd[-1], xd[-2] = xd[-2], xd[-1]
    if trans_y and yn >= 2:
        yd[-1], yd[-2] = yd[-2], yd[-1]
    nb = max(xn, yn) - 2
    batch = _ALPHA[:max(nb, 0)]
    xa = (batch[len(batch) - (xn - 2):] if xn > 2 else '') + ('mk' if xn >= 2 else 'k')
    ya = (batch[len(batch) - (yn - 2):] if yn > 2 else '') + ('kn' if yn >= 2 else 'k')
    oa = batch + ('m' if xn >= 2 else '') + ('n' if yn >= 2 else '')
    req, out, partial = einsum_rule([xa, ya], [xd, yd], oa)
    if trans_x and xn >= 2:
        req[0][-1], req[0][-2] = req[0][-2], req[0][-1]
    if trans_y and yn >= 2:
        req[1][-1], req[1][-2] = req[1][-2], req[1][-1]
    return req, out, partial


def rule_reduce(shape, dm, axis, keepdim):
    n = len(shape)
    ax = _ALPHA[:n]
    red = set(range(n)) if axis is None else {a % n for a in (axis if isinstance(axis, (list, tuple)) else [axis])}
    out = ''.join(('1' if i in red else ax[i]) if keepdim else ('' if i in red else ax[i]) for i in range(n))
    return einsum_rule([ax], [dm], out)


def rule_keep_axes_replicated(shape, dm, axes):
    n = len(shape)
    ax = _ALPHA[:n]
    rep = [ax[a % n] for a in axes]
    return einsum_rule([ax], [dm], ax, rep)


# ------------------------------------------------------------------ differentiable collectives
def _world_group(g):
    return g


def _all_gather_cat(t, group, n, dim):
    t = t.contiguous()
    parts = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts, dim)


def _reduce_scatter_dim(t, group, n, idx, dim):
    t = t.contiguous().clone()
    dist.all_reduce(t, group=group)  # gloo has no reduce_scatter; RCCL: all-reduce = RS + AG anyway for small
    return t.chunk(n, dim)[idx].contiguous()


class _AllGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, group, n, idx, dim):
        ctx.n, ctx.idx, ctx.dim = n, idx, dim
        return _all_gather_cat(t, group, n, dim)

    @staticmethod
    def backward(ctx, g):
        return g.chunk(ctx.n, ctx.dim)[ctx.idx].contiguous(), None, None, None, None


class _Slice(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, group, n, idx, dim):
        ctx.group, ctx.n, ctx.dim = group, n, dim
        return t.chunk(n, dim)[idx].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _all_gather_cat(g, ctx.group, ctx.n, ctx.dim), None, None, None, None


class _AllReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, group, n, avg):
        ctx.n, ctx.avg = n, avg
        out = t.contiguous().clone()
        dist.all_reduce(out, group=group)
        return out / n if avg else out

    @staticmethod
    def backward(ctx, g):
        return (g / ctx.n if ctx.avg else g), None, None, None


class _ReduceScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, group, n, idx, dim):
        ctx.group, ctx.n, ctx.dim = group, n, dim
        return _reduce_scatter_dim(t, group, n, idx, dim)

    @staticmethod
    def backward(ctx, g):
        return _all_gather_cat(g, ctx.group, ctx.n, ctx.dim), None, None, None, None


class _CopyTo(torch.autograd.Function):
    """Identity forward; the gradient is a partial sum over the mesh dim -> all-reduce."""

    @staticmethod
    def forward(ctx, t, group):
        ctx.group = group
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        dist.all_reduce(g, group=ctx.group)
        return g, None


def _recording():
    from ..static.program import recording
    return recording()


def _local_ctx():
    """Local (per-shard) math of a handler: torch functions off — except while a static Program is
    recorded, where the op must reach the recorder (the mode below this one)."""
    return contextlib.nullcontext() if _recording() else torch._C.DisableTorchFunction()


def _apply(fn, t, *extra):
    """``fn.apply(t, *extra)`` — or, while a static Program is recorded (dist.to_static with
    tensor-parallel placements), ONE program node that runs it at replay (the collective and its
    conjugate backward), with the output's meta shape taken from a meta run of the local math."""
    if not _recording():
        return fn.apply(t, *extra)
    from ..static.program import py_node, _paused
    from ..core.tensor import _wrap, _unwrap
    with _paused():
        m = torch.empty(t.shape, dtype=t.dtype, device='meta')
        if fn is _AllGather:
            n, dim = extra[1], extra[3]
            shape = list(t.shape)
            shape[dim] *= n
            out = torch.empty(shape, dtype=t.dtype, device='meta')
        elif fn in (_Slice, _ReduceScatter):
            out = torch.empty_like(m.chunk(extra[1], extra[3])[extra[2]], device='meta')
        else:
            out = m.clone()
    run = lambda x: _wrap(fn.apply(_unwrap(x), *extra))  # noqa: E731
    run._spmd_fn = fn  # Program.reshard_nodes
    return _unwrap(py_node(run, [t], [out])[0])


def _reshard_local(t, mesh, src, dst):
    """Differentiable transition of the local piece ``t`` from placements src to dst."""
    ap = _ap()
    rank = dist.get_rank()
    cur = t
    src = list(src)
    for d in range(mesh.ndim):
        s, p = src[d], dst[d]
        if s == p:
            continue
        grp, ranks = mesh.dim_group(d, rank)
        n, idx = len(ranks), ranks.index(rank)
        if n == 1:
            src[d] = p
            continue
        if isinstance(s, ap.Partial):
            avg = s.reduce_type == ap.ReduceType.kRedAvg
            if isinstance(p, ap.Shard):
                cur = _apply(_ReduceScatter, cur, grp, n, idx, p.dim)
                if avg:
                    cur = cur / n
            else:
                cur = _apply(_AllReduce, cur, grp, n, avg)
                if isinstance(p, ap.Partial):
                    cur = cur if idx == 0 else torch.zeros_like(cur)
        elif isinstance(s, ap.Shard):
            if isinstance(p, ap.Shard):
                cur = _apply(_AllGather, cur, grp, n, idx, s.dim)
                cur = _apply(_Slice, cur, grp, n, idx, p.dim)
            else:
                cur = _apply(_AllGather, cur, grp, n, idx, s.dim)
                if isinstance(p, ap.Partial) and idx != 0:
                    cur = cur * 0
        else:  # Replicate -> Shard / Partial
            if isinstance(p, ap.Shard):
                cur = _apply(_Slice, cur, grp, n, idx, p.dim)
            elif isinstance(p, ap.Partial) and idx != 0:
                cur = cur * 0
        src[d] = p
    return cur


# ------------------------------------------------------------------ op table
_DUNDER_LOCAL = {'__float__', '__int__', '__bool__', '__index__', '__complex__', '__len__', '__repr__',
                 '__format__', '__array__', '__reduce_ex__'}


def _norm_name(func):
    n = getattr(func, '__name__', '')
    return n if n in _DUNDER_LOCAL else n.strip('_')


_EW = {'add', 'sub', 'mul', 'div', 'true_divide', 'subtract', 'multiply', 'divide', 'maximum', 'minimum', 'where',
       'radd', 'rsub', 'rmul', 'rtruediv', 'truediv'}
_UNARY = {'relu', 'gelu', 'silu', 'tanh', 'sigmoid', 'exp', 'neg', 'abs', 'sqrt', 'rsqrt', 'square', 'pow',
          'dropout', 'float', 'bfloat16', 'half', 'to', 'type_as', 'clone', 'contiguous', 'log', 'sin', 'cos',
          'leaky_relu', 'elu', 'softplus', 'scale'}
_LINEAR_UNARY = {'neg', 'float', 'bfloat16', 'half', 'to', 'clone', 'contiguous', 'type_as', 'scale'}
_MATMUL = {'matmul', 'mm', 'bmm'}
_REDUCE = {'sum', 'mean'}
_SOFTMAX = {'softmax', 'log_softmax'}


def _flat_tensors(args):
    return [a for a in args if isinstance(a, torch.Tensor)]


class SpmdMode(TorchFunctionMode):
    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if not any(meta(a) is not None for a in args if isinstance(a, torch.Tensor)) and \
                not any(meta(v) is not None for v in kwargs.values() if isinstance(v, torch.Tensor)):
            return func(*args, **kwargs)
        name = _norm_name(func)
        try:
            handler = _dispatch(name)
        except KeyError:
            return func(*args, **kwargs)
        return handler(func, name, args, kwargs)


def _mesh_of(tensors):
    for t in tensors:
        m = meta(t)
        if m is not None:
            return m[0]
    return None


def _spec(t, mesh):
    m = meta(t)
    if m is None:
        return list(t.shape), [-1] * t.dim(), {}
    _, pl, gs = m
    return gs, dims_mapping(pl, len(gs)), partial_dims(pl)


def _resolve_partial(t, mesh):
    """Partial inputs are all-reduced first (non-linear consumers)."""
    m = meta(t)
    if m is None or not partial_dims(m[1]):
        return t
    ap = _ap()
    src = m[1]
    dst = [ap.Replicate() if isinstance(p, ap.Partial) else p for p in src]
    out = _reshard_local(t, mesh, src, dst)
    return tag(out, mesh, dst, m[2])


def _run(func, args, kwargs, tensor_pos, rule_out, mesh, out_gshape_fn, keep_partial=False):
    """Reshard the tensor args at tensor_pos to the rule's requirements, run, tag the output.
    keep_partial: the op is linear in its inputs, so a Partial input stays Partial (the output
    carries the same partial dims, given in rule_out)."""
    req, out_dm, out_partial = rule_out
    ap = _ap()
    args = list(args)
    active = {d for d in out_dm if d >= 0} | set(out_partial)
    for pos, dm_req in zip(tensor_pos, req):
        t = args[pos]
        m = meta(t)
        src = m[1] if m is not None else [ap.Replicate() for _ in range(mesh.ndim)]
        dst = placements_of(dm_req, partial_dims(src) if keep_partial else {}, mesh.ndim)
        local = _reshard_local(t, mesh, src, dst)
        if t.requires_grad:
            for d in active:
                if d not in dm_req and mesh.shape[d] > 1:
                    grp, _ = mesh.dim_group(d)
                    local = _apply(_CopyTo, local, grp)
        args[pos] = local
    with _local_ctx():
        out = func(*args, **kwargs)
    pl = placements_of(out_dm, {d: ap.ReduceType.kRedSum for d in out_partial}, mesh.ndim)
    if isinstance(out, torch.Tensor):
        tag(out, mesh, pl, out_gshape_fn(out))
    return out


def _gshape(local, dm, mesh):
    return [s * (mesh.shape[dm[i]] if i < len(dm) and dm[i] >= 0 else 1) for i, s in enumerate(local.shape)]


def _h_elementwise(func, name, args, kwargs):
    pos = [i for i, a in enumerate(args) if isinstance(a, torch.Tensor)]
    mesh = _mesh_of([args[i] for i in pos])
    linear = name in ('add', 'sub', 'subtract', 'radd', 'rsub')
    specs = [_spec(args[i], mesh) for i in pos]
    parts = [s[2] for s in specs]
    if linear and len(pos) == 2 and parts[0] and parts[0] == parts[1]:
        # partial + partial along the same mesh dims stays partial (linear op)
        rule = rule_elementwise([s[0] for s in specs], [s[1] for s in specs])
        req, out, _ = rule
        out_partial = set(parts[0])
        return _run(func, args, kwargs, pos, (req, out, out_partial), mesh, lambda o: _gshape(o, out, mesh),
                    keep_partial=True)
    args = list(args)
    for i in pos:
        args[i] = _resolve_partial(args[i], mesh)
    specs = [_spec(args[i], mesh) for i in pos]
    req, out, partial = rule_elementwise([s[0] for s in specs], [s[1] for s in specs])
    return _run(func, args, kwargs, pos, (req, out, partial), mesh, lambda o: _gshape(o, out, mesh))


def _h_unary(func, name, args, kwargs):
    x = args[0]
    mesh = _mesh_of([x])
    if mesh is None:
        return func(*args, **kwargs)
    if name not in _LINEAR_UNARY:
        x = _resolve_partial(x, mesh)
    gs, dm, part = _spec(x, mesh)
    args = (x,) + tuple(args[1:])
    keep = set(part) if name in _LINEAR_UNARY else set()
    return _run(func, args, kwargs, [0], ([dm], dm, keep), mesh, lambda o: _gshape(o, dm, mesh),
                keep_partial=bool(keep))


def _h_matmul(func, name, args, kwargs):
    mesh = _mesh_of(args[:2])
    x, y = _resolve_partial(args[0], mesh), _resolve_partial(args[1], mesh)
    sx, sy = _spec(x, mesh), _spec(y, mesh)
    req, out, partial = rule_matmul([sx[0], sy[0]], [sx[1], sy[1]])
    return _run(func, (x, y) + tuple(args[2:]), kwargs, [0, 1], (req, out, partial), mesh,
                lambda o: _gshape(o, out, mesh))


def _h_linear(func, name, args, kwargs):
    """F.linear(x, W[out, in], b): x @ W^T + b."""
    x, w = args[0], args[1]
    b = args[2] if len(args) > 2 else kwargs.get('bias')
    mesh = _mesh_of([t for t in (x, w, b) if t is not None])
    x, w = _resolve_partial(x, mesh), _resolve_partial(w, mesh)
    sx, sw = _spec(x, mesh), _spec(w, mesh)
    req, out, partial = rule_matmul([sx[0], sw[0]], [sx[1], sw[1]], trans_y=True)
    tensors = [x, w]
    reqs = list(req)
    if b is not None:
        b = _resolve_partial(b, mesh)
        bdm = [out[-1]] if not partial else [-1]
        tensors.append(b)
        reqs.append(bdm)
        if partial:  # bias must be added once: apply it after the partial sum is resolved
            y = _run(func, (x, w, None), {}, [0, 1], (req, out, partial), mesh, lambda o: _gshape(o, out, mesh))
            y = _resolve_partial(y, mesh)
            return y + b
    args2 = tuple(tensors) + tuple(args[3:]) if b is not None else (x, w)
    kw = {k: v for k, v in kwargs.items() if k != 'bias'}
    return _run(func, args2, kw, list(range(len(tensors))), (reqs, out, partial), mesh,
                lambda o: _gshape(o, out, mesh))


def _h_addmm(func, name, args, kwargs):
    """addmm(bias, x, W[in, out]) — the 2-D form paddle's F.linear lowers to: the matmul rule, the
    partial sum resolved, then the (possibly sharded) bias added by the elementwise rule."""
    inp, x, w = args[0], args[1], args[2]
    beta, alpha = kwargs.get('beta', 1), kwargs.get('alpha', 1)
    y = _h_matmul(torch.mm, 'mm', (x, w), {})
    mesh = _mesh_of([y, inp, x, w])
    y = _resolve_partial(y, mesh)
    if alpha != 1:
        y = _h_elementwise(torch.mul, 'mul', (y, alpha), {})
    if beta != 1:
        inp = _h_elementwise(torch.mul, 'mul', (inp, beta), {})
    return _h_elementwise(torch.add, 'add', (y, inp), {})


def _h_sdpa(func, name, args, kwargs):
    """scaled_dot_product_attention(q, k, v [B, H, S, D], attn_mask, ...): batch and head axes may
    stay sharded (q's mapping, k / v / a per-batch or per-head mask follow it); sequence and head
    dims are gathered.  Heads are independent, so every rank attends its own heads exactly."""
    kwargs = dict(kwargs)
    args = list(args)
    if len(args) < 4 and isinstance(kwargs.get('attn_mask'), torch.Tensor):
        args += [None] * (3 - len(args)) + [kwargs.pop('attn_mask')]
    q, k, v = args[0], args[1], args[2]
    mask = args[3] if len(args) > 3 and isinstance(args[3], torch.Tensor) else None
    mesh = _mesh_of([t for t in (q, k, v, mask) if t is not None])
    q, k, v = (_resolve_partial(t, mesh) for t in (q, k, v))
    args[0], args[1], args[2] = q, k, v
    gq, dq, _ = _spec(q, mesh)
    gk, _, _ = _spec(k, mesh)
    nd = len(gq)
    lead = list(dq[:nd - 2]) if nd == 4 and gk[:nd - 2] == gq[:nd - 2] else [-1] * (nd - 2)
    req = [lead + [-1, -1]] * 3
    pos = [0, 1, 2]
    if mask is not None:
        mask = _resolve_partial(mask, mesh)
        args[3] = mask
        gm = _spec(mask, mesh)[0]
        off = nd - len(gm)
        mreq = []
        for i, sz in enumerate(gm):
            j = i + off
            mreq.append(lead[j] if 0 <= j < nd - 2 and sz == gq[j] else -1)
        req.append(mreq)
        pos.append(3)
    gv = _spec(v, mesh)[0]
    out = lead + [-1, -1]
    return _run(func, tuple(args), kwargs, pos, (req, out, set()), mesh, lambda o: list(gq[:-1]) + [gv[-1]])


def _axis_arg(args, kwargs, name='dim'):
    if len(args) > 1 and not isinstance(args[1], torch.dtype):
        return args[1]
    return kwargs.get(name, kwargs.get('axis'))


def _h_reduce(func, name, args, kwargs):
    x = args[0]
    mesh = _mesh_of([x])
    x = _resolve_partial(x, mesh)
    gs, dm, _ = _spec(x, mesh)
    axis = _axis_arg(args, kwargs)
    keep = bool(kwargs.get('keepdim', args[2] if len(args) > 2 and isinstance(args[2], bool) else False))
    req, out, partial = rule_reduce(gs, dm, axis, keep)
    args = (x,) + tuple(args[1:])
    if name == 'mean' and partial:
        # local mean * (local count / global count): a partial SUM of the global mean
        n = len(gs)
        red = range(n) if axis is None else [a % n for a in (axis if isinstance(axis, (list, tuple)) else [axis])]
        scale = 1.0 / math.prod(mesh.shape[dm[a]] for a in red if dm[a] >= 0)
        y = _run(func, args, kwargs, [0], ([dm], out, partial), mesh, lambda o: _gshape(o, out, mesh))
        m = meta(y)
        y2 = y * scale
        return tag(y2, m[0], m[1], m[2])
    return _run(func, args, kwargs, [0], ([dm], out, partial), mesh, lambda o: _gshape(o, out, mesh))


def _h_keep_axes(axes_fn):
    def h(func, name, args, kwargs):
        x = args[0]
        mesh = _mesh_of([x])
        x = _resolve_partial(x, mesh)
        gs, dm, _ = _spec(x, mesh)
        axes = axes_fn(gs, args, kwargs)
        req, out, partial = rule_keep_axes_replicated(gs, dm, axes)
        rest = list(args[1:])
        pos = [0]
        # layer_norm weight / bias: replicate (their axes are the normalised ones)
        for i, a in enumerate(rest):
            if isinstance(a, torch.Tensor):
                rest[i] = _resolve_partial(a, mesh)
                pos.append(i + 1)
                req.append([-1] * a.dim())
        return _run(func, (x,) + tuple(rest), kwargs, pos, (req, out, partial), mesh,
                    lambda o: _gshape(o, out, mesh))
    return h


def _softmax_axes(gs, args, kwargs):
    d = args[1] if len(args) > 1 and isinstance(args[1], int) else kwargs.get('dim', -1)
    return [d if d is not None else -1]


def _layernorm_axes(gs, args, kwargs):
    ns = args[1] if len(args) > 1 else kwargs.get('normalized_shape')
    k = len(ns) if isinstance(ns, (list, tuple, torch.Size)) else 1
    return list(range(len(gs) - k, len(gs)))


def _h_transpose(func, name, args, kwargs):
    x = args[0]
    mesh = _mesh_of([x])
    gs, dm, part = _spec(x, mesh)
    n = len(gs)
    if name == 'permute':
        perm = list(args[1]) if len(args) == 2 and isinstance(args[1], (list, tuple)) else [int(a) for a in args[1:]]
    elif name == 't':
        perm = [1, 0] if n == 2 else list(range(n))
    else:
        a, b = args[1] % n, args[2] % n
        perm = list(range(n))
        perm[a], perm[b] = perm[b], perm[a]
    out = [dm[p] for p in perm]
    return _run(func, args, kwargs, [0], ([dm], out, set(part)), mesh, lambda o: _gshape(o, out, mesh),
                keep_partial=True)


def _h_reshape(func, name, args, kwargs):
    """Sharded dims survive a reshape when they keep their prefix (the dims before them are
    unchanged) and their size, or become the leading factor of a merged output dim; otherwise the
    input is replicated first (reference reshape.cc builds the general dim-transform)."""
    x = args[0]
    mesh = _mesh_of([x])
    gs, dm, part = _spec(x, mesh)
    shp = args[1] if len(args) == 2 and isinstance(args[1], (list, tuple, torch.Size)) else list(args[1:])
    shp = list(shp)
    total = math.prod(gs)
    if -1 in shp:
        k = shp.index(-1)
        rest = math.prod(v for i, v in enumerate(shp) if i != k)
        shp[k] = total // max(rest, 1)
    out = [-1] * len(shp)
    ok = True
    for i, d in enumerate(dm):
        if d < 0:
            continue
        pre = math.prod(gs[:i])
        j, acc = 0, 1
        while j < len(shp) and acc < pre:
            acc *= shp[j]
            j += 1
        if acc != pre or j >= len(shp):
            ok = False
        elif shp[j] % gs[i] == 0:  # kept, or the leading factor of a merge
            out[j] = d
        elif gs[i] % shp[j] == 0 and shp[j] % mesh.shape[d] == 0:  # split: shard the leading factor
            out[j] = d
        else:
            ok = False
    if not ok:
        ap = _ap()
        src = meta(x)[1]
        dst = [ap.Replicate() if isinstance(p, ap.Shard) else p for p in src]
        x = tag(_reshard_local(x, mesh, src, dst), mesh, dst, gs)
        dm = [-1] * len(gs)
        out = [-1] * len(shp)
    # local target shape: divide sharded output dims
    local_shape = [v // (mesh.shape[out[i]] if out[i] >= 0 else 1) for i, v in enumerate(shp)]
    with _local_ctx():
        y = func(x, local_shape) if name != 'view' else x.view(local_shape)
    ap = _ap()
    return tag(y, mesh, placements_of(out, {d: ap.ReduceType.kRedSum for d in part}, mesh.ndim), shp)


def _h_embedding(func, name, args, kwargs):
    ids, w = args[0], args[1]
    mesh = _mesh_of([ids, w])
    si, sw = _spec(ids, mesh), _spec(w, mesh)
    n = len(si[0])
    ia = _ALPHA[:n]
    req, out, partial = einsum_rule([ia, 'vh'], [si[1], sw[1]], ia + 'h', replicate_axes=('v',))
    return _run(func, args, kwargs, [0, 1], (req, out, partial), mesh, lambda o: _gshape(o, out, mesh))


def _h_cross_entropy(func, name, args, kwargs):
    logits, label = args[0], args[1]
    mesh = _mesh_of([logits, label])
    logits = _resolve_partial(logits, mesh)
    sl, sb = _spec(logits, mesh), _spec(label, mesh)
    n = len(sl[0])
    la = _ALPHA[:n]
    lb = la[:len(sb[0])]
    red = kwargs.get('reduction', 'mean')
    out_axes = la[:-1] if red == 'none' else ''
    req, out, partial = einsum_rule([la, lb], [sl[1], sb[1]], out_axes, replicate_axes=(la[-1],))
    if red == 'mean' and partial:
        kw = dict(kwargs)
        kw['reduction'] = 'sum'
        y = _run(func, (logits, label) + tuple(args[2:]), kw, [0, 1], (req, out, partial), mesh, lambda o: [])
        cnt = math.prod(sb[0])
        m = meta(y)
        return tag(y / cnt, m[0], m[1], m[2])
    return _run(func, (logits, label) + tuple(args[2:]), kwargs, [0, 1], (req, out, partial), mesh,
                lambda o: _gshape(o, out, mesh))


def _dispatch(name):
    if name in _DUNDER_LOCAL:
        raise KeyError(name)
    if name in _EW:
        return _h_elementwise
    if name in _UNARY:
        return _h_unary
    if name in _MATMUL:
        return _h_matmul
    if name == 'linear':
        return _h_linear
    if name == 'addmm':
        return _h_addmm
    if name == 'scaled_dot_product_attention':
        return _h_sdpa
    if name in _REDUCE:
        return _h_reduce
    if name in _SOFTMAX:
        return _h_keep_axes(_softmax_axes)
    if name == 'layer_norm':
        return _h_keep_axes(_layernorm_axes)
    if name in ('transpose', 'permute', 't'):
        return _h_transpose
    if name in ('reshape', 'view'):
        return _h_reshape
    if name == 'embedding':
        return _h_embedding
    if name == 'cross_entropy':
        return _h_cross_entropy
    raise KeyError(name)


_mode = [None]


def enable():
    """Install the SPMD mode (idempotent; called by shard_tensor)."""
    if _mode[0] is None:
        m = SpmdMode()
        m.__enter__()
        _mode[0] = m


def disable():
    if _mode[0] is not None:
        _mode[0].__exit__(None, None, None)
        _mode[0] = None
