"""paddle.static.nn (reference: python/paddle/static/nn/common.py fc/conv2d/batch_norm/embedding...,
control_flow.py cond:…, while_loop, case, switch_case).

Layer helpers create their parameters eagerly (that is the startup program) and apply the
dygraph functional, which the recorder captures.  Control flow traces each branch / the loop
body into a sub-op-list once; the executor picks the branch (or iterates) at run time.
"""
import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from .. import nn as _nn
from ..nn import functional as F
from .program import default_main_program, Node, Ref, _to_record, _vid_of, _paused


def _meta_like(t):
    with _paused():
        return torch.empty_like(t, device='meta')


def _act(x, act):
    if act is None:
        return x
    return getattr(F, act)(x)


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    outs = []
    for xi in xs:
        shp = xi.shape
        in_f = 1
        for d in shp[num_flatten_dims:]:
            in_f *= d
        lin = _nn.Linear(in_f, size, weight_attr=weight_attr, bias_attr=bias_attr)
        h = xi if len(shp) == num_flatten_dims + 1 else xi.reshape(list(shp[:num_flatten_dims]) + [in_f])
        outs.append(lin(h))
    out = outs[0]
    for o in outs[1:]:
        out = out + o
    return _act(out, activation)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1, param_attr=None,  # noqa: A002
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCHW"):
    cin = input.shape[1] if data_format == 'NCHW' else input.shape[-1]
    conv = _nn.Conv2D(cin, num_filters, filter_size, stride, padding, dilation, groups, weight_attr=param_attr,
                      bias_attr=bias_attr, data_format=data_format)
    return _act(conv(input), act)


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,  # noqa: A002
                     groups=1, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format='NCHW'):
    cin = input.shape[1] if data_format == 'NCHW' else input.shape[-1]
    conv = _nn.Conv2DTranspose(cin, num_filters, filter_size, stride, padding, groups=groups, dilation=dilation,
                               weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    return _act(conv(input), act)


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,  # noqa: A002
               data_layout='NCHW', in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=True, use_global_stats=False):
    c = input.shape[1] if data_layout == 'NCHW' else input.shape[-1]
    bn = _nn.BatchNorm(c, momentum=momentum, epsilon=epsilon, param_attr=param_attr, bias_attr=bias_attr,
                       data_layout=data_layout, use_global_stats=use_global_stats)
    if is_test:
        bn.eval()
    return _act(bn(input), act)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,  # noqa: A002
               act=None, name=None):
    shape = input.shape[begin_norm_axis:]
    ln = _nn.LayerNorm(shape, epsilon=epsilon, weight_attr=param_attr if scale else False,
                       bias_attr=bias_attr if shift else False)
    return _act(ln(input), act)


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,  # noqa: A002
              dtype='float32'):
    emb = _nn.Embedding(size[0], size[1], padding_idx=padding_idx, weight_attr=param_attr)
    return emb(input)


def prelu(x, mode='all', param_attr=None, data_format="NCHW", name=None):
    n = 1 if mode == 'all' else (x.shape[1] if data_format == 'NCHW' else x.shape[-1])
    return _nn.PReLU(n, weight_attr=param_attr, data_format=data_format)(x)


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout='NCHW', in_place=False, name=None,  # noqa: A002
              moving_mean_name=None, moving_variance_name=None, do_model_average_for_mean_and_var=True,
              slot_dim=-1, sync_stats=False, summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    """Reference static/nn/common.py data_norm (CTR feature normalisation): persistent batch
    statistics batch_size / batch_sum / batch_square_sum (init 1e4 / 0 / 1e4, like the reference),
    y = (x - sum/size) * sqrt(size / square_sum); the statistics decay by summary_decay_rate and
    absorb each training batch (the reference updates them in its backward)."""
    from ..core.tensor import Parameter
    C = input.shape[-1] if data_layout == 'NHWC' or len(input.shape) == 2 else input.shape[1]

    def stat(v):
        p = Parameter(torch.full([C], float(v)), trainable=False)
        p.stop_gradient = True
        return p
    size, ssum, sq = stat(1e4), stat(0.0), stat(1e4)
    mean = ssum / size
    scale = (size / sq).sqrt()
    y = (input - mean) * scale
    if enable_scale_and_shift:
        w = _nn.Layer().create_parameter([C], default_initializer=_nn.initializer.Constant(1.0))
        b = _nn.Layer().create_parameter([C], default_initializer=_nn.initializer.Constant(0.0), is_bias=True)
        y = y * w + b
    if not _is_static(input):  # dygraph: update the statistics with this batch
        with torch.no_grad():
            x = _unwrap(input).reshape(-1, C).float()
            for p, v in ((size, torch.full([C], float(x.shape[0]))), (ssum, x.sum(0)), (sq, (x * x).sum(0))):
                p._t.mul_(summary_decay_rate).add_(v.to(p._t.device, p._t.dtype))
    return _act(y, act)


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None, data_layout='NCHW',  # noqa: A002
               name=None):
    c = input.shape[1] if data_layout == 'NCHW' else input.shape[-1]
    gn = _nn.GroupNorm(groups, c, epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr,
                       data_format=data_layout)
    return _act(gn(input), act)


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):  # noqa: A002
    c = input.shape[1]
    cls = {3: _nn.InstanceNorm1D, 4: _nn.InstanceNorm2D, 5: _nn.InstanceNorm3D}[len(input.shape)]
    return cls(c, epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr)(input)


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1, param_attr=None,  # noqa: A002
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCDHW"):
    cin = input.shape[1] if data_format == 'NCDHW' else input.shape[-1]
    conv = _nn.Conv3D(cin, num_filters, filter_size, stride, padding, dilation, groups, weight_attr=param_attr,
                      bias_attr=bias_attr, data_format=data_format)
    return _act(conv(input), act)


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,  # noqa: A002
                     groups=1, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format='NCDHW'):
    cin = input.shape[1] if data_format == 'NCDHW' else input.shape[-1]
    conv = _nn.Conv3DTranspose(cin, num_filters, filter_size, stride, padding, groups=groups, dilation=dilation,
                               weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    return _act(conv(input), act)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    """out_k = x W_k y^T + b_k (reference static/nn/common.py bilinear_tensor_product)."""
    bl = _nn.Bilinear(x.shape[-1], y.shape[-1], size, weight_attr=param_attr, bias_attr=bias_attr)
    return _act(bl(x, y), act)


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    sn = _nn.SpectralNorm(list(weight.shape), axis=dim, power_iters=power_iters, epsilon=eps)
    return sn(weight)


def deform_conv2d(x, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1,
                  deformable_groups=1, im2col_step=1, weight_attr=None, bias_attr=None, name=None):
    from ..vision.ops import DeformConv2D
    dc = DeformConv2D(x.shape[1], num_filters, filter_size, stride, padding, dilation, deformable_groups, groups,
                      weight_attr=weight_attr, bias_attr=bias_attr)
    return dc(x, offset, mask)


def sparse_embedding(input, size, padding_idx=None, is_test=False, entry=None, table_class="MemorySparseTable",  # noqa: A002
                     param_attr=None, dtype='float32', slot=None):
    """Parameter-server sparse table lookup; on one process a dense embedding of the same shape."""
    return embedding(input, size, is_sparse=True, padding_idx=padding_idx, param_attr=param_attr, dtype=dtype)


def row_conv(input, future_context_size, param_attr=None, act=None):  # noqa: A002
    """Lookahead convolution (reference static/nn/common.py row_conv, DeepSpeech2): out[t] =
    sum_{j=0..k} x[t+j] * W[j] per feature, within each sequence of a LoD input or along the time
    axis of a padded [B, T, D] input."""
    D = input.shape[-1]
    w = _nn.Layer().create_parameter([future_context_size + 1, D], attr=param_attr)
    if not _is_static(input) and input.__dict__.get('_lod') is not None:
        from . import sequence as S
        lod = S.get_lod(input)
        out = _wrap(S.row_conv_lod(_unwrap(input).reshape(-1, D), lod, _unwrap(w)))
        return _act(S.with_lod(out, lod), act)
    x = _unwrap(input)
    T = x.shape[1]
    xp = torch.nn.functional.pad(x, (0, 0, 0, future_context_size))
    out = sum(xp[:, j:j + T] * _unwrap(w)[j] for j in range(future_context_size + 1))
    return _act(_wrap(out), act)


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None,  # noqa: A002
        num_neg_samples=None, name=None, sampler='uniform', custom_dist=None, seed=0, is_sparse=False):
    """Noise-contrastive estimation loss (reference static/nn/common.py nce / nce_op.h): for each
    example the true class and num_neg_samples sampled classes are scored with a logistic model
    o = sigmoid(x·w_c + b_c); cost = -log(o_true / (o_true + k q)) - sum log(k q / (o_neg + k q)),
    q = the sampler's probability of the class.  Returns [batch, 1]."""
    k = 10 if num_neg_samples is None else int(num_neg_samples)
    D = input.shape[-1]
    layer = _nn.Layer()
    w = layer.create_parameter([num_total_classes, D], attr=param_attr)
    b = layer.create_parameter([num_total_classes, 1], attr=bias_attr, is_bias=True)
    x = _unwrap(input)
    lab = _unwrap(label).reshape(x.shape[0], -1).long()
    B = x.shape[0]
    g = torch.Generator(device='cpu').manual_seed(int(seed))
    if sampler == 'uniform':
        q_all = torch.full([num_total_classes], 1.0 / num_total_classes)
        neg = torch.randint(0, num_total_classes, (B, k), generator=g)
    elif sampler == 'log_uniform':
        r = torch.arange(num_total_classes, dtype=torch.float64)
        q_all = (torch.log((r + 2) / (r + 1)) / np.log(num_total_classes + 1)).float()
        neg = torch.multinomial(q_all, B * k, replacement=True, generator=g).reshape(B, k)
    elif sampler == 'custom_dist':
        q_all = torch.as_tensor(np.asarray(custom_dist), dtype=torch.float32)
        neg = torch.multinomial(q_all, B * k, replacement=True, generator=g).reshape(B, k)
    else:
        raise ValueError(f"unknown sampler {sampler}")
    neg = neg.to(x.device)
    q_all = q_all.to(x.device, x.dtype)
    W, bb = _unwrap(w), _unwrap(b).reshape(-1)

    def score(cls):
        return torch.sigmoid((x.unsqueeze(1) * W[cls]).sum(-1) + bb[cls])
    o_t, o_n = score(lab), score(neg)
    kq_t, kq_n = k * q_all[lab], k * q_all[neg]
    cost = -torch.log(o_t / (o_t + kq_t)).sum(1) - torch.log(kq_n / (o_n + kq_n)).sum(1)
    if sample_weight is not None:
        cost = cost * _unwrap(sample_weight).reshape(-1)
    return _wrap(cost.reshape(B, 1))


def static_pylayer(forward_fn, inputs, backward_fn=None, name=None):
    """Reference static/nn/static_pylayer.py: run forward_fn on inputs; with backward_fn the
    gradient of the outputs w.r.t. the inputs is backward_fn(*output_grads)."""
    if backward_fn is None:
        return forward_fn(*inputs)

    class _SPL(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *ts):
            with torch.no_grad():
                outs = forward_fn(*[_wrap(t) for t in ts])
            ctx.multi = isinstance(outs, (list, tuple))
            outs = outs if ctx.multi else [outs]
            return tuple(_unwrap(o) for o in outs) if ctx.multi else _unwrap(outs[0])

        @staticmethod
        def backward(ctx, *gs):
            res = backward_fn(*[_wrap(g) for g in gs])
            res = res if isinstance(res, (list, tuple)) else [res]
            return tuple(None if r is None else _unwrap(r) for r in res)
    out = _SPL.apply(*[_unwrap(t) for t in inputs])
    return [_wrap(o) for o in out] if isinstance(out, tuple) else _wrap(out)


# ----------------------------------------------------------------- control flow
def _trace(fn, args=()):
    """Records what ``fn(*args)`` does into a separate op list; returns (nodes, outputs)."""
    prog = default_main_program()
    saved = prog.nodes
    prog.nodes = []
    try:
        out = fn(*args)
    finally:
        sub = prog.nodes
        prog.nodes = saved
    return sub, out


def _flat(out):
    if out is None:
        return []
    if isinstance(out, (list, tuple)):
        r = []
        for o in out:
            r.extend(_flat(o))
        return r
    return [out]


def _refs(prog, outs):
    res = []
    for o in outs:
        t = _unwrap(o)
        if isinstance(t, torch.Tensor) and t.is_meta:
            res.append(Ref(_vid_of(prog, t)))
        else:
            res.append(_to_record(prog, t))
    return res


def _restructure(like, flat):
    it = iter(flat)

    def go(o):
        if isinstance(o, (list, tuple)):
            return type(o)(go(x) for x in o)
        if o is None:
            return None
        return next(it)
    return go(like)


def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    """Both branches are traced; the executor runs the one ``pred`` selects."""
    prog = default_main_program()
    if not (isinstance(_unwrap(pred), torch.Tensor) and _unwrap(pred).is_meta):
        # eager predicate (dygraph or constant): plain Python branch
        p = bool(_unwrap(pred).item()) if isinstance(pred, Tensor) else bool(pred)
        fn = true_fn if p else false_fn
        return fn() if fn is not None else None
    t_nodes, t_out = _trace(true_fn) if true_fn is not None else ([], None)
    f_nodes, f_out = _trace(false_fn) if false_fn is not None else ([], None)
    t_flat, f_flat = _flat(t_out), _flat(f_out)
    if len(t_flat) != len(f_flat):
        raise ValueError("true_fn and false_fn must return the same structure")
    outs = []
    metas = []
    for a in t_flat:
        m = _meta_like(_unwrap(a))
        outs.append(prog._new_value(m))
        metas.append(_wrap(m))
    prog.nodes.append(Node('cond', None, [Ref(_vid_of(prog, _unwrap(pred)))], {
        'branches': (t_nodes, _refs(prog, t_flat), f_nodes, _refs(prog, f_flat))}, outs))
    return _restructure(t_out, metas) if t_out is not None else None


def while_loop(cond, body, loop_vars, is_test=False, name=None):  # noqa: A002
    prog = default_main_program()
    lv = list(loop_vars)
    if not any(isinstance(_unwrap(v), torch.Tensor) and _unwrap(v).is_meta for v in lv):
        while bool(_unwrap(cond(*lv)).item()):
            out = body(*lv)
            lv = list(out) if isinstance(out, (list, tuple)) else [out]
        return lv
    # fresh values for the carried variables inside the traced bodies
    carried = []
    cvids = []
    for v in lv:
        m = _meta_like(_unwrap(v))
        cvids.append(prog._new_value(m))
        carried.append(_wrap(m))
    c_nodes, c_out = _trace(cond, carried)
    b_nodes, b_out = _trace(body, carried)
    b_flat = _flat(b_out)
    outs = []
    metas = []
    for v in lv:
        m = _meta_like(_unwrap(v))
        outs.append(prog._new_value(m))
        metas.append(_wrap(m))
    prog.nodes.append(Node('while', None, _refs(prog, lv), {
        'carried': cvids, 'cond': (c_nodes, _refs(prog, [c_out])[0]), 'body': (b_nodes, _refs(prog, b_flat))}, outs))
    return metas


def case(pred_fn_pairs, default=None, name=None):
    def build(pairs):
        if not pairs:
            return default() if default is not None else None
        (p, fn), rest = pairs[0], pairs[1:]
        if not rest and default is None:
            return fn()
        return cond(p, fn, lambda: build(rest))
    return build(list(pred_fn_pairs))


def switch_case(branch_index, branch_fns, default=None, name=None):
    items = list(branch_fns.items()) if isinstance(branch_fns, dict) else (
        list(branch_fns) if isinstance(branch_fns[0], (list, tuple)) else list(enumerate(branch_fns)))
    pairs = [(branch_index == int(k), fn) for k, fn in items]
    return case(pairs, default if default is not None else items[-1][1])


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    from .program import py_node
    xs = x if isinstance(x, (list, tuple)) else [x]
    outs = out if isinstance(out, (list, tuple)) else [out]
    res = py_node(func, xs, [_meta_like(_unwrap(o)) for o in outs])
    return res if isinstance(out, (list, tuple)) else res[0]


# ----------------------------------------------------------------- LoD sequence ops (static/sequence.py)
def _is_static(x):
    return isinstance(x, Tensor) and x._t.device.type == 'meta'


def _seq(fn, tensors, out_rows_like=None, out_cols=None, n_out=1):
    """Runs a sequence op eagerly, or records it as a py-node inside a static Program (the LoD of
    the fed tensors reaches it through the Executor)."""
    if not any(_is_static(t) for t in tensors if isinstance(t, Tensor)):
        return fn(*tensors)
    from .program import SENTINELS
    t0 = _unwrap(tensors[0])
    cols = list(t0.shape[1:]) if out_cols is None else list(out_cols)
    with _paused():
        metas = [torch.empty([SENTINELS[0]] + cols, dtype=t0.dtype, device='meta') for _ in range(n_out)]
    res = py_func(lambda *ts: fn(*ts), list(tensors), [_wrap(m) for m in metas] if n_out > 1 else _wrap(metas[0]))
    return res


def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):  # noqa: A002
    from . import sequence as S
    return _seq(lambda x: S.sequence_pool(x, pool_type, is_test, pad_value), [input])


def sequence_first_step(input):  # noqa: A002
    return sequence_pool(input, 'first')


def sequence_last_step(input):  # noqa: A002
    return sequence_pool(input, 'last')


def sequence_softmax(input, use_cudnn=False, name=None):  # noqa: A002
    from . import sequence as S
    return _seq(S.sequence_softmax, [input])


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=True, padding_start=None,  # noqa: A002
                  bias_attr=None, param_attr=None, act=None, name=None):
    from . import sequence as S
    if _is_static(input):
        D = input.shape[-1]
        lin = _nn.Linear(filter_size * D, num_filters, weight_attr=param_attr, bias_attr=bias_attr)
        ps = -int(filter_size // 2) if padding_start is None else padding_start

        def run(x):
            ctx = S._context_rows(_unwrap(x).reshape(x.shape[0], D), S.get_lod(x), filter_size, ps)
            out = lin(_wrap(ctx))
            return S.with_lod(_act(out, act), S.get_lod(x))
        return _seq(run, [input], out_cols=[num_filters])
    return S.sequence_conv(input, num_filters, filter_size, filter_stride, padding, padding_start, bias_attr,
                           param_attr, act, name)


def sequence_slice(input, offset, length, name=None):  # noqa: A002
    from . import sequence as S
    return _seq(lambda x, o, l: S.sequence_slice(x, o, l), [input, offset, length])


def sequence_expand(x, y, ref_level=-1, name=None):
    from . import sequence as S
    return _seq(lambda a, b: S.sequence_expand(a, b, ref_level), [x, y])


def sequence_expand_as(x, y, name=None):
    from . import sequence as S
    return _seq(S.sequence_expand_as, [x, y])


def sequence_pad(x, pad_value, maxlen=None, name=None):
    from . import sequence as S
    if _is_static(x):
        return _seq(lambda a, p: S.sequence_pad(a, p, maxlen), [x, pad_value], n_out=2)
    return S.sequence_pad(x, pad_value, maxlen)


def sequence_unpad(x, length, name=None):
    from . import sequence as S
    return _seq(S.sequence_unpad, [x, length], out_cols=list(x.shape[2:]))


def sequence_reshape(input, new_dim):  # noqa: A002
    from . import sequence as S
    return _seq(lambda a: S.sequence_reshape(a, new_dim), [input], out_cols=[new_dim])


def sequence_scatter(input, index, updates, name=None):  # noqa: A002
    from . import sequence as S
    return _seq(S.sequence_scatter, [input, index, updates])


def sequence_enumerate(input, win_size, pad_value=0, name=None):  # noqa: A002
    from . import sequence as S
    return _seq(lambda a: S.sequence_enumerate(a, win_size, pad_value), [input], out_cols=[win_size])
