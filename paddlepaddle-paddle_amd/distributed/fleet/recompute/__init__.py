"""Activation recomputation (reference: python/paddle/distributed/fleet/recompute/recompute.py,
recompute_hybrid.py).

``recompute(fn, *args)`` drops the activations of ``fn`` in forward and re-runs it in backward
(RNG state restored so dropout masks match).  On MI355X (288 GB HBM) recompute is usually a
memory/perf trade NOT needed for ≤13B models at moderate micro-batches; it is provided for
long-sequence / giant-model configs.
"""
import torch
import torch.utils.checkpoint as _ckpt

from ....core.tensor import Tensor, _wrap, _unwrap


def _flatten(obj, out):
    if isinstance(obj, Tensor):
        out.append(obj._t)
        return ('T', len(out) - 1)
    if isinstance(obj, (list, tuple)):
        return (type(obj), [_flatten(o, out) for o in obj])
    return ('C', obj)


def _rebuild(spec, flat):
    kind, v = spec
    if kind == 'T':
        return _wrap(flat[v])
    if kind == 'C':
        return v
    return kind(_rebuild(s, flat) for s in v)


def _static_checkpoint(function, args, kwargs):
    """recompute() while a static Program records: the segment's ops go into a 'checkpoint' node
    whose body the Executor runs under torch's non-reentrant checkpoint (static/executor.py
    _exec_checkpoint) — the recorded program recomputes the segment in backward, as the eager
    path does (reference: the static recompute pass, distributed/passes/auto_parallel_recompute.py)."""
    from ....static import program as P
    prog = P.default_main_program()
    flat = []
    _flatten(list(args) + list(kwargs.values()), flat)
    ins = []
    for t in flat:
        tt = t._t if isinstance(t, Tensor) else t
        if isinstance(tt, torch.Tensor) and tt.is_meta and id(tt) in prog._val:
            ins.append(P.Ref(prog._val[id(tt)]))
    saved, prog.nodes = prog.nodes, []
    try:
        res = function(*args, **kwargs)
    finally:
        body, prog.nodes = prog.nodes, saved
    outs = []
    _flatten(res, outs)
    out_vids = []
    for t in outs:
        tt = t._t if isinstance(t, Tensor) else t
        if isinstance(tt, torch.Tensor) and id(tt) in prog._val:
            out_vids.append(prog._val[id(tt)])
    params = [c for c in getattr(prog, '_const_owner', {}).values() if c is not None and not c.stop_gradient]
    prog.nodes.append(P.Node('checkpoint', None, ins, {'body': body, 'params': bool(params)}, out_vids,
                             {'stage': P._STAGE[0]}))
    return res


def recompute(function, *args, **kwargs):
    from ....static.program import recording
    if recording():
        kwargs.pop('preserve_rng_state', None)
        kwargs.pop('use_reentrant', None)
        kwargs.pop('offload_indices', None)
        return _static_checkpoint(function, args, kwargs)
    preserve = kwargs.pop('preserve_rng_state', True)
    kwargs.pop('use_reentrant', None)
    offload = kwargs.pop('offload_indices', None)  # noqa: F841
    flat = []
    spec = _flatten(list(args), flat)
    out_spec = {}

    def run(*ts):
        a = _rebuild(spec, list(ts))
        res = function(*a, **kwargs)
        outs = []
        out_spec['s'] = _flatten(res, outs)
        return tuple(outs)
    if not torch.is_grad_enabled():
        return function(*args, **kwargs)
    outs = _ckpt.checkpoint(run, *flat, use_reentrant=False, preserve_rng_state=preserve)
    return _rebuild(out_spec['s'], list(outs))


def recompute_sequential(ctx, functions, *args, **kwargs):
    segments = ctx.get('segments', 1) if isinstance(ctx, dict) else 1
    preserve = ctx.get('preserve_rng_state', True) if isinstance(ctx, dict) else True
    layers = list(functions.children()) if hasattr(functions, 'children') else list(functions)
    seg = max(len(layers) // max(segments, 1), 1)
    x = args[0] if len(args) == 1 else args

    def run_seg(lo, hi):
        def f(inp):
            for l in layers[lo:hi]:
                inp = l(inp)
            return inp
        return f
    for lo in range(0, len(layers), seg):
        x = recompute(run_seg(lo, min(lo + seg, len(layers))), x, preserve_rng_state=preserve)
    return x


def recompute_hybrid(ctx, function, *args, **kwargs):
    return recompute(function, *args, **kwargs)
