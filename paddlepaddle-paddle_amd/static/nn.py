"""paddle.static.nn (reference: python/paddle/static/nn/common.py fc/conv2d/batch_norm/embedding...,
control_flow.py cond:…, while_loop, case, switch_case).

Layer helpers create their parameters eagerly (that is the startup program) and apply the
dygraph functional, which the recorder captures.  Control flow traces each branch / the loop
body into a sub-op-list once; the executor picks the branch (or iterates) at run time.
"""
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


def data_norm(input, *a, **k):  # noqa: A002
    return F.batch_norm(input, None, None, training=True) if False else layer_norm(input)


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


def sequence_pool(*a, **k):
    raise NotImplementedError("LoD sequence ops are not supported; use padded tensors with masks")
