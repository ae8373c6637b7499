"""Executor (reference: python/paddle/base/executor.py:1182 Executor.run; global_scope,
scope_guard; compiler.py CompiledProgram/BuildStrategy).

``run`` interprets a recorded Program on real device tensors: feeds bind data values, sentinel
extents in recorded integer arguments are specialised to the fed shapes, parameters are read
live, and backward/update nodes drive torch autograd + our optimizers.  Programs without a
backward node run under no_grad.
"""
import contextlib

import numpy as np
import torch

from ..core.tensor import Tensor, _wrap
from . import symbolic as _sym
from .program import (Program, Ref, Const, default_main_program, default_startup_program, SENTINELS, _paused,
                      _vid_of)


class Scope:
    def __init__(self):
        self.vars = {}

    def var(self, name):
        return self.vars.setdefault(name, _ScopeVar(name))

    def find_var(self, name):
        from .program import default_main_program as _m
        prog = _m()
        if name in prog.named_vars or name in self.vars:
            return self.vars.setdefault(name, _ScopeVar(name))
        for p in prog.all_parameters():
            if p.name == name:
                v = _ScopeVar(name)
                v._t = p
                return v
        return None


class _ScopeVar:
    def __init__(self, name):
        self.name = name
        self._t = None

    def get_tensor(self):
        return self._t

    def set(self, value, place=None):
        self._t = value


_scope = [Scope()]


def global_scope():
    return _scope[-1]


@contextlib.contextmanager
def scope_guard(scope):
    _scope.append(scope)
    try:
        yield
    finally:
        _scope.pop()


class BuildStrategy:
    def __init__(self):
        self.fuse_elewise_add_act_ops = False
        self.fuse_bn_act_ops = False
        self.fuse_all_reduce_ops = True
        self.enable_inplace = True
        self.memory_optimize = True
        self.build_cinn_pass = False
        self.debug_graphviz_path = ''


class ExecutionStrategy:
    def __init__(self):
        self.num_threads = 1
        self.num_iteration_per_drop_scope = 100


class CompiledProgram:
    def __init__(self, program_or_graph, build_strategy=None):
        self.program = program_or_graph
        self.build_strategy = build_strategy or BuildStrategy()

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None, share_vars_from=None,
                           places=None):
        return self


class _SymEnv(dict):
    """Symbol index -> fed extent (an unfed symbol keeps its carrier extent)."""

    def __init__(self, smap):
        super().__init__()
        self.smap = smap

    def __missing__(self, i):
        return self.smap.get(SENTINELS[i], SENTINELS[i])


def _subst_int(v, smap, prog=None):
    """A recorded int at run time: a SymInt's expression (or a value-table entry's) evaluated with
    the fed extents; other ints unchanged.  Programs without a value table (loaded from the
    pre-symbolic format) re-specialise by factoring the carrier primes out."""
    if isinstance(v, bool) or v == 0 or not smap:
        return int(v) if isinstance(v, _sym.SymInt) else v
    if isinstance(v, _sym.SymInt):
        return v.expr.eval(_SymEnv(smap))
    if prog is not None and getattr(prog, '_symbolic', False):
        e = prog._symvals.get(v)
        return e.eval(_SymEnv(smap)) if e is not None else v
    out, rest = 1, v
    hit = False
    for s in SENTINELS:
        while rest % s == 0 and s in smap:
            rest //= s
            out *= smap[s]
            hit = True
    return rest * out if hit else v


def _resolve(prog, obj, env, smap, dev):
    if isinstance(obj, Ref):
        return env[obj.vid]
    if isinstance(obj, Const):
        owner = prog._const_owner.get(obj.cid) if hasattr(prog, '_const_owner') else None
        # a parameter resolves to its live storage (static.amp O2 / set_state_dict may replace it)
        return owner._t if owner is not None else prog.consts[obj.cid]
    if isinstance(obj, bool) or obj is None:
        return obj
    if isinstance(obj, int):
        return _subst_int(obj, smap, prog)
    if isinstance(obj, torch.device):
        return dev if obj.type == 'meta' else obj
    if isinstance(obj, str) and obj == 'meta':
        return dev
    if isinstance(obj, torch.Size):
        return torch.Size([_subst_int(x, smap, prog) for x in obj])
    if isinstance(obj, tuple) and hasattr(obj, '_fields'):
        return type(obj)(*[_resolve(prog, o, env, smap, dev) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_resolve(prog, o, env, smap, dev) for o in obj)
    if isinstance(obj, dict):
        return {k: _resolve(prog, v, env, smap, dev) for k, v in obj.items()}
    if isinstance(obj, slice):
        return slice(_resolve(prog, obj.start, env, smap, dev), _resolve(prog, obj.stop, env, smap, dev),
                     _resolve(prog, obj.step, env, smap, dev))
    return obj


def _bind(env, outs, val):
    if outs is None:
        return
    if isinstance(outs, int):
        env[outs] = val
        return
    for o, v in zip(outs, val):
        _bind(env, o, v)


def _feed_tensor(v, dt, dev):
    if isinstance(v, Tensor):
        t = v._t
    elif isinstance(v, torch.Tensor):
        t = v
    else:
        a = np.asarray(v)
        t = torch.from_numpy(a) if a.dtype != np.object_ else torch.tensor(a.tolist())
    return t.to(device=dev, dtype=dt)


_SUBS = {'map': None}  # target substitutions of the running replay (static.amp fp8: ops/fp8.py)


# per-node timing of the running replay (paddle.cost_model.CostModel.profile_measure): None, or a
# list receiving (node index, op name, milliseconds); device work is synchronised per node
_PROFILE = {'rec': None}


def _op_name(n):
    t = n.target
    return getattr(t, '__name__', None) or type(t).__name__ if n.kind in ('torch', 'py') else n.kind


def _exec(prog, nodes, env, smap, dev):
    rec = _PROFILE['rec']
    if rec is None:
        return _exec_nodes(prog, nodes, env, smap, dev)
    import time
    sync = (lambda: torch.cuda.synchronize(dev)) if dev is not None and torch.device(dev).type == 'cuda' else \
        (lambda: None)
    for i, n in enumerate(nodes):
        sync()
        t0 = time.perf_counter()
        _exec_nodes(prog, [n], env, smap, dev)
        sync()
        rec.append((len(rec), _op_name(n), (time.perf_counter() - t0) * 1e3))


_GEMM_SUBS = {}


def _gemm_subs():
    """Recorded torch GEMM targets (matmul / mm / bmm / addmm / einsum / linear) -> the hand-written
    MFMA GEMM routing of ops/matmul.py (torch itself for CPU / fp32 / out-of-contract shapes)."""
    if not _GEMM_SUBS:
        from ..ops import matmul as _hm
        _GEMM_SUBS.update(_hm.static_substitutions())
    return _GEMM_SUBS


_ZB = {'map': None}  # zero-bubble static pipeline: weight GEMMs with deferred dW (static/pipeline.py)


def _exec_nodes(prog, nodes, env, smap, dev):
    subs = _SUBS['map']
    gsubs = _gemm_subs()
    zb = _ZB['map']
    for n in nodes:
        if n.kind == 'torch':
            args = _resolve(prog, n.args, env, smap, dev)
            kwargs = _resolve(prog, n.kwargs, env, smap, dev)
            if n.meta.get('factory') and 'device' in kwargs and kwargs['device'] is None:
                kwargs['device'] = dev
            fn = subs.get(n.target, n.target) if subs else n.target
            try:
                fn = zb.get(fn, fn) if zb is not None else fn
                fn = gsubs.get(fn, fn)
            except TypeError:  # unhashable target
                pass
            _bind(env, n.outs, fn(*args, **kwargs))
        elif n.kind == 'minimize':
            loss = env[n.args[0].vid]
            if hasattr(n.target, '_static_minimize_exec'):  # static.amp: loss scaling / skip-on-inf
                n.target._static_minimize_exec(loss)
            else:
                loss.backward()
                n.target.step()
                from .amp import release_grads
                release_grads(n.target)
        elif n.kind == 'backward':
            loss = env[n.args[0].vid]
            loss.backward()
            params = n.kwargs['params']
            _bind(env, n.outs, [p._t.grad if p._t.grad is not None else torch.zeros_like(p._t) for p in params])
            for p in params:
                p._t.grad = None
        elif n.kind == 'grad':
            ts = _resolve(prog, n.args[0], env, smap, dev)
            xs = _resolve(prog, n.args[1], env, smap, dev)
            gs = _resolve(prog, n.args[2], env, smap, dev)
            gs = [g if g is not None else torch.ones_like(t) for g, t in zip(gs, ts)]
            res = torch.autograd.grad(ts, xs, gs, retain_graph=True, allow_unused=True)
            _bind(env, n.outs, [r if r is not None else torch.zeros_like(x) for r, x in zip(res, xs)])
        elif n.kind == 'py':
            args = _resolve(prog, n.args, env, smap, dev)
            ins = []
            for a in args:
                if isinstance(a, torch.Tensor):
                    w = _wrap(a)
                    if id(a) in _LOD:  # LoD of a fed / produced sequence tensor (static/sequence.py)
                        w.__dict__['_lod'] = _LOD[id(a)][1]
                    ins.append(w)
                else:
                    ins.append(a)
            out = n.target(*ins)
            out = out if isinstance(out, (list, tuple)) else [out]
            for o in out:
                if isinstance(o, Tensor) and o.__dict__.get('_lod') is not None:
                    _LOD[id(o._t)] = (o._t, o.__dict__['_lod'])  # keep the tensor alive with its id
            _bind(env, n.outs, [o._t if isinstance(o, Tensor) else o for o in out])
        elif n.kind == 'cond':
            t_nodes, t_refs, f_nodes, f_refs = n.kwargs['branches']
            take = bool(_resolve(prog, n.args[0], env, smap, dev).reshape(-1)[0].item())
            nodes_, refs = (t_nodes, t_refs) if take else (f_nodes, f_refs)
            _exec(prog, nodes_, env, smap, dev)
            _bind(env, n.outs, [_resolve(prog, r, env, smap, dev) for r in refs])
        elif n.kind == 'while':
            cur = [_resolve(prog, r, env, smap, dev) for r in n.args]
            c_nodes, c_ref = n.kwargs['cond']
            b_nodes, b_refs = n.kwargs['body']
            while True:
                for vid, v in zip(n.kwargs['carried'], cur):
                    env[vid] = v
                _exec(prog, c_nodes, env, smap, dev)
                if not bool(_resolve(prog, c_ref, env, smap, dev).reshape(-1)[0].item()):
                    break
                _exec(prog, b_nodes, env, smap, dev)
                cur = [_resolve(prog, r, env, smap, dev) for r in b_refs]
            _bind(env, n.outs, cur)
        elif n.kind == 'checkpoint':
            _exec_checkpoint(prog, n, env, smap, dev)
        else:
            raise RuntimeError(f"unknown node kind {n.kind}")


def _checkpoint_outs(prog, n):
    """Values of a checkpoint body that anything outside it reads (declared outputs, later
    nodes, fetchable variables): computed once, from the finished program."""
    outs = n.meta.get('live_outs')
    if outs is not None:
        return outs
    body_ids = {id(b) for b in n.kwargs['body']}
    produced = set()
    from .ir_passes import _outs_of, _refs_in
    for b in n.kwargs['body']:
        produced.update(_outs_of(b.outs, []))
    used = set()

    def scan(nodes):
        for m in nodes:
            if id(m) in body_ids:
                continue
            r = []
            _refs_in(m.args, r)
            _refs_in(m.kwargs, r)
            used.update(r)
            for k in ('body', 'branches', 'cond'):
                sub = m.kwargs.get(k) if isinstance(m.kwargs, dict) else None
                if isinstance(sub, list):
                    scan(sub)
    scan(prog.nodes)
    for var in prog.named_vars.values():
        vid = prog._val.get(id(getattr(var, '_t', None)))
        if vid is not None:
            used.add(vid)
    outs = [v for v in _outs_of(n.outs, []) if v in produced]
    outs += sorted((produced & used) - set(outs))
    n.meta['live_outs'] = outs
    return outs


def _exec_checkpoint(prog, n, env, smap, dev):
    """A recompute segment (fleet.recompute under static recording): the body's activations are
    not kept for backward — torch's non-reentrant checkpoint re-runs the body in backward."""
    from torch.utils import checkpoint as _ckpt
    ins = [_resolve(prog, r, env, smap, dev) for r in n.args]
    outs = _checkpoint_outs(prog, n)
    body = n.kwargs['body']

    def run(*xs):
        env2 = dict(env)
        for r, x in zip(n.args, xs):
            env2[r.vid] = x
        _exec_nodes(prog, body, env2, smap, dev)
        return tuple(env2[v] for v in outs)
    if torch.is_grad_enabled() and any(isinstance(x, torch.Tensor) and x.requires_grad for x in ins) or \
            torch.is_grad_enabled() and n.kwargs.get('params'):
        res = _ckpt.checkpoint(run, *ins, use_reentrant=False, preserve_rng_state=True)
    else:
        res = run(*ins)
    for v, t in zip(outs, res):
        env[v] = t


_LOD = {}  # id(torch tensor) -> (tensor, level-1 offsets) for LoD values of the running replay


def _pipeline_policy(prog):
    for n in reversed(prog.nodes):
        if n.kind == 'minimize':
            return n.target if getattr(n.target, 'pipeline', None) is not None else None
    return None


def _run_pipelined(prog, feed, dev, pol):
    """One pipeline-parallel training step (static/pipeline.py) on this rank's stage."""
    from .pipeline import run_pipeline
    from .amp import autocast_context

    def run_forward(nodes, env, feed_m):
        smap = {}
        _bind_feeds(prog, feed_m, dev, env, smap)
        with _paused(), autocast_context(prog, dev) as subs:
            prev, _SUBS['map'] = _SUBS['map'], subs
            try:
                _exec(prog, nodes, env, smap, dev)
            finally:
                _SUBS['map'] = prev
    _LOD.clear()
    return run_pipeline(prog, feed, dev, pol, pol.pipeline, run_forward)


def run_program(prog, feed, dev, grad=None, fetch=None):
    """Interpret ``prog``; returns the value env.  ``fetch``: the value ids the caller will read
    (lets the dead-code / common-subexpression passes drop and merge everything else)."""
    pol = _pipeline_policy(prog)
    if pol is not None and (grad is None or grad):
        return _run_pipelined(prog, feed, dev, pol)
    env = {}
    smap = {}
    _LOD.clear()
    _bind_feeds(prog, feed, dev, env, smap)
    needs_grad = grad if grad is not None else any(n.kind in ('minimize', 'backward', 'grad') for n in prog.nodes)
    ctx = contextlib.nullcontext() if needs_grad else torch.no_grad()
    from .amp import autocast_context
    from .ir_passes import ir_nodes
    nodes = ir_nodes(prog, dev, fetch)  # the fusion-pass rewrite (static/ir_passes.py) on GPU programs
    with _paused(), ctx, autocast_context(prog, dev) as subs:
        prev, _SUBS['map'] = _SUBS['map'], subs
        try:
            _exec(prog, nodes, env, smap, dev)
        finally:
            _SUBS['map'] = prev
    return env


def _bind_feeds(prog, feed, dev, env, smap):
    feed = feed or {}
    for name, (vid, shape, dt) in prog.feeds.items():
        if name not in feed:
            continue
        t = _feed_tensor(feed[name], dt, dev)
        if len(shape) == t.dim():
            for i, s in enumerate(shape):
                if s == -1:
                    sent = SENTINELS[i]
                    if sent in smap and smap[sent] != t.shape[i]:
                        raise ValueError(f"feed '{name}' dim {i} = {t.shape[i]} conflicts with another feed's {smap[sent]}")
                    smap[sent] = t.shape[i]
                elif s != t.shape[i]:
                    raise ValueError(f"feed '{name}' expects shape {shape}, got {list(t.shape)}")
        env[vid] = t
        lod = feed[name].__dict__.get('_lod') if isinstance(feed[name], Tensor) else None
        if lod is not None:
            _LOD[id(t)] = (t, lod)


class Executor:
    def __init__(self, place=None):
        from ..core.place import to_device
        self.place = place
        self._dev = to_device(place)

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name='feed', fetch_var_name='fetch', scope=None,
            return_numpy=True, use_program_cache=False, return_merged=True, use_prune=False):
        if isinstance(program, CompiledProgram):
            program = program.program
        if program is None:
            program = default_main_program()
        if not isinstance(program, Program):
            raise TypeError("Executor.run expects a static Program")
        if program is default_startup_program() or (not program.nodes and not program.feeds):
            return []  # parameters are initialised when their layers are created
        from ..decomposition import decomp as _decomp
        if _decomp._prim_config['prim_enabled'] and not getattr(program, '_prim_decomposed', False):
            _decomp.decompose(program, [])  # incubate.autograd.enable_prim(): run on primitive ops
            program._prim_decomposed = True
        fetch_list = fetch_list if fetch_list is not None else []
        if not isinstance(fetch_list, (list, tuple)):
            fetch_list = [fetch_list]
        env = run_program(program, feed, self._dev, fetch=self._fetch_vids(program, fetch_list))
        out = []
        for f in fetch_list:
            t = self._fetch(program, env, f)
            if return_numpy:
                t = t.detach()
                out.append((t.float() if t.dtype == torch.bfloat16 else t).cpu().numpy())
            else:
                out.append(_wrap(t))
        return out

    @staticmethod
    def _fetch_vids(program, fetch_list):
        """Value ids of the fetch targets (None when one cannot be resolved before the run)."""
        vids = []
        for f in fetch_list:
            if isinstance(f, str):
                f = program.named_vars.get(f)
                if f is None:
                    continue  # a parameter name: read from its live storage, not the env
            tt = f._t if isinstance(f, Tensor) else f
            if not isinstance(tt, torch.Tensor) or not tt.is_meta:
                continue
            vid = program._val.get(id(tt))
            if vid is None:
                return None
            vids.append(vid)
        return tuple(sorted(set(vids)))

    @staticmethod
    def _fetch(program, env, f):
        if isinstance(f, str):
            if f in program.named_vars:
                f = program.named_vars[f]
            else:
                for p in program.all_parameters():
                    if p.name == f:
                        return p._t
                raise KeyError(f"fetch target '{f}' not found in program")
        tt = f._t if isinstance(f, Tensor) else f
        if tt.is_meta:
            return env[_vid_of(program, tt)]
        return tt

    def close(self):
        pass

    def train_from_dataset(self, program=None, dataset=None, scope=None, thread=0, debug=False, fetch_list=None,
                           fetch_info=None, print_period=100, fetch_handler=None):
        """Run ``program`` over every batch of a fleet dataset (reference base/executor.py
        train_from_dataset): the dataset parses its slot files into feeds of its ``use_var``
        variables; ``fetch_list`` values are printed every ``print_period`` batches (labelled by
        ``fetch_info``) and handed to ``fetch_handler.handler`` when given.  Returns the last
        batch's fetches."""
        return self._run_from_dataset(program, dataset, fetch_list, fetch_info, print_period, fetch_handler, debug)

    def infer_from_dataset(self, program=None, dataset=None, scope=None, thread=0, debug=False, fetch_list=None,
                           fetch_info=None, print_period=100, fetch_handler=None):
        """As train_from_dataset, for a program without an optimizer (reference infer_from_dataset)."""
        return self._run_from_dataset(program, dataset, fetch_list, fetch_info, print_period, fetch_handler, debug)

    def _run_from_dataset(self, program, dataset, fetch_list, fetch_info, print_period, fetch_handler, debug):
        if dataset is None:
            raise RuntimeError("dataset is needed and should be initialized")
        fetch_list = list(fetch_list or [])
        fetch_info = list(fetch_info or [getattr(f, 'name', str(i)) for i, f in enumerate(fetch_list)])
        last = []
        for bi, feed in enumerate(dataset._iter_batches()):
            last = self.run(program, feed=feed, fetch_list=fetch_list) if fetch_list else self.run(program, feed=feed)
            if fetch_list and print_period and (bi + 1) % print_period == 0:
                print(", ".join(f"{n}: {v}" for n, v in zip(fetch_info, last)), flush=True)
            if fetch_handler is not None and fetch_list:
                fetch_handler.handler(dict(zip(fetch_info, last)))
        return last


ParallelExecutor = Executor
