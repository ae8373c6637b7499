"""Static-graph programs (reference: python/paddle/base/framework.py Program/Block/Variable,
program_guard, default_main_program; python/paddle/static/input.py data, InputSpec).

Design: a ``Program`` is a recorded op list (a small IR), not a protobuf desc.  While static
mode is on, a ``TorchFunctionMode`` records every tensor operation whose inputs derive from a
static ``Variable``.  Variables carry *meta* tensors (shape/dtype only, no memory), so building
a program for a 1.3B model costs nothing.  Dynamic dims (``None``/-1) are symbols
(static/symbolic.py): their meta tensors carry large-prime carrier extents, shape reads of program
values return ``SymInt``s that carry a DimExpr through Python shape arithmetic (``B*S``,
``arange(S)``), and the Executor evaluates the recorded expressions with the fed extents — so user
code that reads ``x.shape`` and reshapes still runs at any feed shape, while plain integer
constants are never touched.

Real tensors touched by a recorded op (parameters, buffers, captured constants) are kept by
reference (``Const``), so optimizer updates made at run time are seen by later runs.
``Executor.run`` interprets the op list on real device tensors (our HIP kernels run inside
the recorded torch ops' implementations or via recorded paddle ops).
"""
import contextlib
import itertools

import torch
from torch.overrides import TorchFunctionMode

from ..core.tensor import Tensor, _wrap
from . import symbolic as _sym

# one sentinel extent per dynamic-dim position (dim 0 = batch, dim 1 = sequence, ...): the six
# largest primes below 2^20, so an unrelated recorded integer is a multiple of one with odds of
# about 1e-6 (meta tensors hold no memory, so the large extents cost nothing; three dynamic dims
# times a 10^4 feature dim stay far inside int64 numel)
SENTINELS = (1048573, 1048571, 1048559, 1048549, 1048517, 1048507)

# pipeline stage of the ops being recorded (static.device_guard('gpu:N') -> N; None outside a guard)
_STAGE = [None]
_SENT_SET = set(SENTINELS)


class Ref:
    """Reference to a program value (output of a node or a fed data variable)."""
    __slots__ = ('vid',)

    def __init__(self, vid):
        self.vid = vid

    def __repr__(self):
        return f"%{self.vid}"


class Const:
    """Reference to a real tensor captured at build time (parameter / buffer / constant)."""
    __slots__ = ('cid',)

    def __init__(self, cid):
        self.cid = cid

    def __repr__(self):
        return f"$c{self.cid}"


class Node:
    __slots__ = ('kind', 'target', 'args', 'kwargs', 'outs', 'meta')

    def __init__(self, kind, target, args, kwargs, outs, meta=None):
        self.kind, self.target, self.args, self.kwargs, self.outs = kind, target, args, kwargs, outs
        self.meta = meta or {}

    def __repr__(self):
        name = getattr(self.target, '__name__', str(self.target))
        return f"{self.outs} = {self.kind}:{name}{tuple(self.args)}"


def _has_sentinel(v, prog=None):
    """Does v (an op argument) depend on a dynamic dim?  SymInts do; a plain int does when the
    program's value table holds it (a SymInt of that value escaped through ``int()`` /
    ``operator.index``) — or, for programs loaded without a value table, when a carrier prime
    divides it (the pre-symbolic rule)."""
    if isinstance(v, bool):
        return False
    if isinstance(v, _sym.SymInt):
        return True
    if isinstance(v, int):
        if v == 0:
            return False
        if prog is not None and getattr(prog, '_symbolic', False):
            return v in prog._symvals
        return any(v % s == 0 for s in SENTINELS)
    if isinstance(v, (list, tuple, torch.Size)):
        return any(_has_sentinel(x, prog) for x in v)
    return False


# shape reads of program values answer in SymInts (static/symbolic.py)
_SHAPE_FUNCS = {torch.Tensor.size, torch.Tensor.numel, torch.Tensor.stride, torch.Tensor.shape.__get__}


def _symbolic_shape(out):
    if isinstance(out, torch.Size):
        return torch.Size([_sym.symbolize(d, SENTINELS) for d in out])
    if isinstance(out, tuple):
        return tuple(_sym.symbolize(d, SENTINELS) for d in out)
    if isinstance(out, int):
        return _sym.symbolize(out, SENTINELS)
    return out


class Block:
    def __init__(self, program, idx=0):
        self.program = program
        self.idx = idx

    @property
    def ops(self):
        return self.program.nodes

    def all_parameters(self):
        return self.program.all_parameters()

    def var(self, name):
        return self.program.var(name)

    @property
    def vars(self):
        return dict(self.program.named_vars)

    def create_var(self, name=None, shape=None, dtype='float32', **kw):
        return data(name or f"tmp_{len(self.program.named_vars)}", shape or [1], dtype)


class Program:
    _ids = itertools.count()

    def __init__(self):
        self.nodes = []
        self.consts = {}        # cid -> real tensor
        self._const_ids = {}    # id(real tensor) -> cid
        self._meta_twins = {}   # cid -> meta twin
        self._vid = itertools.count()
        self._val = {}          # id(meta tensor) -> vid
        self._keep = []         # keeps meta tensors alive so ids stay unique
        self.feeds = {}         # name -> (vid, shape with -1, dtype)
        self.named_vars = {}    # name -> Tensor (Variable)
        self.random_seed = 0
        self._id = next(Program._ids)
        self._blocks = [Block(self)]
        self._for_test = False
        self._symbolic = True   # dynamic dims are symbols (static/symbolic.py)
        self._symvals = {}      # value table: SymInt values that escaped through int() -> DimExpr

    # ---- structure
    def global_block(self):
        return self._blocks[0]

    def block(self, i):
        return self._blocks[i]

    @property
    def blocks(self):
        return self._blocks

    def current_block(self):
        return self._blocks[0]

    def num_blocks(self):
        return 1

    def all_parameters(self):
        from ..core.tensor import Parameter
        return [t for t in self._params()]

    def _params(self):
        out = []
        for cid, t in self.consts.items():
            p = self._const_owner.get(cid) if hasattr(self, '_const_owner') else None
            if p is not None:
                out.append(p)
        return out

    def list_vars(self):
        return list(self.named_vars.values())

    def var(self, name):
        return self.named_vars[name]

    def clone(self, for_test=False):
        p = Program.__new__(Program)
        p.__dict__.update(self.__dict__)
        p.nodes = [n for n in self.nodes if not (for_test and n.kind in ('backward', 'minimize', 'grad'))]
        p._id = next(Program._ids)
        p._blocks = [Block(p)]
        p._for_test = for_test
        return p

    def __repr__(self):
        lines = [f"Program(id={self._id}, {len(self.nodes)} ops, feeds={list(self.feeds)})"]
        lines += ["  " + repr(n) for n in self.nodes[:200]]
        return '\n'.join(lines)

    __str__ = __repr__

    def to_string(self, throw_on_error=False, with_details=False):
        return repr(self)

    def dist_attr(self, value):
        """(process_mesh, placements, global_shape) of a value recorded under SPMD propagation
        (DistModel programs), None for a value with no dist attribute. ``value``: a Ref, a value
        id or a recorded Variable."""
        if isinstance(value, Ref):
            value = value.vid
        if isinstance(value, int):
            for t in self._keep:
                if self._val.get(id(t)) == value:
                    return getattr(t, '_pd_dist', None)
            return None
        t = getattr(value, '_t', value)
        a = getattr(t, '_pd_dist', None)
        if a is None and isinstance(t, torch.Tensor):
            twin = self._meta_twins.get(self._const_ids.get(id(t)))
            a = getattr(twin, '_pd_dist', None)
        return a

    def reshard_nodes(self):
        """The collective nodes SPMD propagation inserted (all-gather / reduce-scatter / ...)."""
        return [n for n in self.nodes if getattr(n.target, '_spmd_fn', None) is not None]

    # ---- recording helpers
    def _new_value(self, meta_t):
        vid = next(self._vid)
        self._val[id(meta_t)] = vid
        self._keep.append(meta_t)
        return vid

    def _const(self, t, owner=None):
        cid = self._const_ids.get(id(t))
        if cid is None:
            cid = len(self.consts)
            self.consts[cid] = t
            self._const_ids[id(t)] = cid
            if not hasattr(self, '_const_owner'):
                self._const_owner = {}
            self._const_owner[cid] = owner
            with _paused():
                twin = torch.empty_like(t, device='meta')
            if t.requires_grad and t.is_leaf:
                twin.requires_grad_(True)
            self._meta_twins[cid] = twin
        return cid


# ----------------------------------------------------------------- program stack / mode
_main = [Program()]
_startup = [Program()]


def default_main_program():
    return _main[-1]


def default_startup_program():
    return _startup[-1]


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    _main.append(main_program)
    if startup_program is not None:
        _startup.append(startup_program)
    try:
        yield
    finally:
        _main.pop()
        if startup_program is not None:
            _startup.pop()


def _paddle_param_of(t):
    from ..core.tensor import _PARAMS
    p = _PARAMS.get(id(t))
    if p is not None and p._t is t:
        return p
    return None


class _Recorder(TorchFunctionMode):
    """Records tensor ops that consume static values into the current main program."""

    def __init__(self):
        super().__init__()
        self.paused = 0

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in _SHAPE_FUNCS and args and isinstance(args[0], torch.Tensor) and args[0].is_meta:
            # shape reads (also while paused): carrier extents come back as SymInts
            prog = default_main_program()
            out = func(*args, **kwargs)
            with _sym.recording_table(prog._symvals):
                return _symbolic_shape(out)
        if self.paused:
            return func(*args, **kwargs)
        prog = default_main_program()
        metas = []
        _scan(args, metas)
        _scan(kwargs, metas)
        dev_meta = any(isinstance(v, torch.device) and v.type == 'meta' for v in kwargs.values()) or \
            kwargs.get('device') == 'meta'
        static_input = any(t.is_meta and id(t) in prog._val for t in metas)
        forced = getattr(prog, '_force_record_ids', None)  # decomposition: ops on captured params
        if forced and not static_input:
            static_input = any(id(t) in forced for t in metas)
        if not static_input and not dev_meta and not (not metas and (_has_sentinel(list(args), prog) or
                                                                    _has_sentinel(list(kwargs.values()), prog))):
            if any(t.is_meta for t in metas):
                return func(*args, **kwargs)  # meta work unrelated to this program
            return func(*args, **kwargs)
        # map inputs: program values -> Ref, real tensors -> Const (+ meta twin for shape inference)
        rec_args = _to_record(prog, args)
        rec_kwargs = _to_record(prog, kwargs)
        meta_args = _to_meta(prog, args)
        meta_kwargs = _to_meta(prog, kwargs)
        factory = not metas
        if factory:
            meta_kwargs = dict(meta_kwargs)
            if 'device' in _factory_kw(func):
                meta_kwargs['device'] = 'meta'
        out = func(*meta_args, **meta_kwargs)
        if not _tree_has_tensor(out):
            return out
        out = _metaize(out)
        outs = _register_outs(prog, out)
        prog.nodes.append(Node('torch', func, rec_args, rec_kwargs, outs, {'factory': factory, 'stage': _STAGE[0]}))
        return out


def _factory_kw(func):
    name = getattr(func, '__name__', '')
    if name in ('zeros', 'ones', 'empty', 'full', 'arange', 'rand', 'randn', 'randint', 'eye', 'linspace',
                'logspace', 'tensor', 'as_tensor', 'zeros_like', 'ones_like', 'empty_like', 'full_like',
                'randn_like', 'rand_like', 'tril_indices', 'triu_indices', 'randperm', 'normal', 'scalar_tensor'):
        return ('device',)
    return ()


def _scan(obj, out):
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _scan(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _scan(o, out)


def _tree_has_tensor(obj):
    if isinstance(obj, torch.Tensor):
        return True
    if isinstance(obj, (list, tuple)):
        return any(_tree_has_tensor(o) for o in obj)
    return False


def _metaize(obj):
    if isinstance(obj, torch.Tensor):
        return obj if obj.is_meta else obj.to('meta')
    if isinstance(obj, tuple) and hasattr(obj, '_fields'):
        return type(obj)(*[_metaize(o) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_metaize(o) for o in obj)
    return obj


def _register_outs(prog, out):
    if isinstance(out, torch.Tensor):
        vid = prog._val.get(id(out))
        if vid is None:
            vid = prog._new_value(out)
        return vid
    if isinstance(out, (list, tuple)):
        return [_register_outs(prog, o) for o in out]
    return None


def _to_record(prog, obj):
    if isinstance(obj, torch.Tensor):
        if obj.is_meta:
            vid = prog._val.get(id(obj))
            if vid is None:
                raise RuntimeError("a meta tensor not produced by this program was used in a static op")
            return Ref(vid)
        return Const(prog._const(obj, _paddle_param_of(obj)))
    if isinstance(obj, tuple) and hasattr(obj, '_fields'):
        return type(obj)(*[_to_record(prog, o) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_record(prog, o) for o in obj)
    if isinstance(obj, dict):
        return {k: _to_record(prog, v) for k, v in obj.items()}
    return obj


def _to_meta(prog, obj):
    if isinstance(obj, torch.Tensor):
        if obj.is_meta:
            return obj
        return prog._meta_twins[prog._const(obj, _paddle_param_of(obj))]
    if isinstance(obj, tuple) and hasattr(obj, '_fields'):
        return type(obj)(*[_to_meta(prog, o) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_meta(prog, o) for o in obj)
    if isinstance(obj, dict):
        return {k: _to_meta(prog, v) for k, v in obj.items()}
    return obj


_recorder = [None]


def _start_recording():
    if _recorder[0] is None:
        r = _Recorder()
        r.__enter__()
        _recorder[0] = r


def _stop_recording():
    r = _recorder[0]
    if r is not None:
        r.__exit__(None, None, None)
        _recorder[0] = None


@contextlib.contextmanager
def _paused():
    r = _recorder[0]
    if r is not None:
        r.paused += 1
    try:
        yield
    finally:
        if r is not None:
            r.paused -= 1


def recording():
    return _recorder[0] is not None and not _recorder[0].paused


def _recording_table():
    return default_main_program()._symvals if _recorder[0] is not None else None


_sym._GETTER[0] = _recording_table


# ----------------------------------------------------------------- data / InputSpec
def _dtype(d):
    from ..core.dtype import to_torch_dtype
    return to_torch_dtype(d)


def _static_shape(shape):
    return [(-1 if (s is None or s < 0) else int(s)) for s in shape]


def _sentinel_shape(shape):
    return [SENTINELS[i] if (s is None or s < 0) else int(s) for i, s in enumerate(shape)]


def data(name, shape, dtype=None, lod_level=0):
    """A feed slot of the current main program (shape entries None/-1 are dynamic)."""
    prog = default_main_program()
    dt = _dtype(dtype or 'float32')
    with _paused():
        t = torch.empty(_sentinel_shape(shape), dtype=dt, device='meta')
    vid = prog._new_value(t)
    prog.feeds[name] = (vid, _static_shape(shape), dt)
    v = _wrap(t)
    v._name = name
    v.__dict__['_lod_level'] = int(lod_level or 0)
    prog.named_vars[name] = v
    return v


class InputSpec:
    def __init__(self, shape, dtype='float32', name=None, stop_gradient=False):
        self.shape = list(shape) if shape is not None else []
        self.dtype = dtype
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(tensor.shape, str(tensor.dtype).replace('paddle.', ''), name or getattr(tensor, 'name', None))

    @classmethod
    def from_numpy(cls, ndarray, name=None):
        return cls(list(ndarray.shape), str(ndarray.dtype), name)

    def batch(self, batch_size):
        return InputSpec([batch_size] + self.shape, self.dtype, self.name)

    def unbatch(self):
        return InputSpec(self.shape[1:], self.dtype, self.name)

    def __repr__(self):
        return f"InputSpec(shape={tuple(self.shape)}, dtype={self.dtype}, name={self.name})"

    def __eq__(self, other):
        return isinstance(other, InputSpec) and (self.shape, str(self.dtype), self.name) == \
            (other.shape, str(other.dtype), other.name)

    def __hash__(self):
        return hash((tuple(self.shape), str(self.dtype), self.name))


def is_static_value(t):
    tt = t._t if isinstance(t, Tensor) else t
    return isinstance(tt, torch.Tensor) and tt.is_meta


def static_shape(t):
    """Tensor.shape in static mode: sentinel extents reported as -1 (reference semantics)."""
    return [(-1 if d in _SENT_SET else d) for d in t.shape]


@contextlib.contextmanager
def name_scope(prefix=None):
    yield



# ----------------------------------------------------------------- backward / optimizer nodes
def _vid_of(prog, t):
    tt = t._t if isinstance(t, Tensor) else t
    vid = prog._val.get(id(tt))
    if vid is None:
        raise ValueError("not a value of the current program")
    return vid


def _static_minimize(opt, loss, parameters=None, no_grad_set=None):
    """optimizer.minimize(loss) in static mode: appends a backward+update node; parameters
    default to every trainable parameter the program reads."""
    prog = default_main_program()
    if parameters is not None:
        params = list(parameters)
    elif opt._parameter_list:
        params = list(opt._parameter_list)
    else:
        params = [p for p in prog.all_parameters() if not p.stop_gradient]
    if no_grad_set:
        skip = {id(p) for p in no_grad_set}
        params = [p for p in params if id(p) not in skip]
    if not opt._parameter_list:
        opt._add_param_group({'params': params})
        opt._parameter_list = list(params)
    prog.nodes.append(Node('minimize', opt, [Ref(_vid_of(prog, loss))], {}, None))
    return None, [(p, None) for p in params]


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None,
                    distop_context=None):
    """Appends a backward node; returns [(param, grad_var)] whose grad vars can be fetched."""
    prog = default_main_program()
    params = list(parameter_list) if parameter_list is not None else \
        [p for p in prog.all_parameters() if not p.stop_gradient]
    outs = []
    grads = []
    for p in params:
        with _paused():
            g = torch.empty_like(p._t, device='meta')
        outs.append(prog._new_value(g))
        gv = _wrap(g)
        gv._name = (p.name or 'param') + '@GRAD'
        prog.named_vars[gv._name] = gv
        grads.append(gv)
    prog.nodes.append(Node('backward', None, [Ref(_vid_of(prog, loss))], {'params': params}, outs))
    return list(zip(params, grads))


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    prog = default_main_program()
    targets = targets if isinstance(targets, (list, tuple)) else [targets]
    inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    tg = target_gradients if target_gradients is not None else [None] * len(targets)
    tg = tg if isinstance(tg, (list, tuple)) else [tg]

    def ref(t):
        tt = t._t
        return Ref(_vid_of(prog, t)) if tt.is_meta else Const(prog._const(tt, _paddle_param_of(tt)))
    outs, res = [], []
    for x in inputs:
        with _paused():
            g = torch.empty_like(x._t, device='meta')
        outs.append(prog._new_value(g))
        res.append(_wrap(g))
    prog.nodes.append(Node('grad', None, [[ref(t) for t in targets], [ref(x) for x in inputs],
                                          [ref(g) if g is not None else None for g in tg]], {}, outs))
    return res


def py_node(fn, inputs, out_metas):
    """Records an eagerly-executed Python callable (control flow, py_func) as one node."""
    prog = default_main_program()
    rec = _to_record(prog, [x._t if isinstance(x, Tensor) else x for x in inputs])
    outs = [prog._new_value(m) for m in out_metas]
    prog.nodes.append(Node('py', fn, rec, {}, outs, {'stage': _STAGE[0]}))
    return [_wrap(m) for m in out_metas]
