"""Dygraph -> static conversion of tensor-dependent Python control flow.

Reference: python/paddle/jit/dy2static/ — ``transformers/ifelse_transformer.py``,
``transformers/loop_transformer.py``, ``transformers/logical_transformer.py``,
``transformers/return_transformer.py``, ``convert_operators.py`` (convert_ifelse:242,
convert_while_loop:48, convert_logical_and/or/not), ``convert_call_func.py`` (convert_call).

The eager path never needs this: ``to_static`` functions run dygraph code directly on the HIP
kernels, and a Python ``if`` on an eager tensor just reads the value.  Conversion matters only
when a function is RECORDED into a static Program (``concrete_program``, ``jit.save``), where
tensors are meta ``Variable``s with no value — there a Python ``if x.mean() > 0`` has to become
a ``cond`` node and ``while i < n`` a ``while`` node that the executor evaluates per call.

How (one AST pass per function, cached per code object):

* ``if``   -> both branches become local functions of the names they assign; the statement
  becomes ``names = _jst.convert_ifelse(test, true_fn, false_fn, values, names, False)``.
  An ``if`` whose branch ends in ``return`` takes the rest of the block as its ``else`` and
  becomes ``return _jst.convert_ifelse(..., True)`` (early return).
* ``while`` -> ``names = _jst.convert_while(cond_fn, body_fn, values, names)``.
* ``for v in range(...)`` -> ``_jst.convert_for_range``.
* ``a and b`` / ``a or b`` / ``not a`` / ``x if c else y`` -> lazy ``_jst.convert_logical_*`` /
  ``convert_ifexp``.
* calls -> ``_jst.convert_call(f)(...)``: user functions and user ``Layer.forward``s reached from
  a converted function are converted too.

At run time every ``convert_*`` checks whether its predicate is a static Variable: if not, it
runs the plain Python statement (so dygraph semantics are untouched); if so it records the
``cond`` / ``while`` node through ``static.nn.cond`` machinery.  Branch outputs are merged per
variable: tensors on both sides become node outputs, a Python number facing a tensor becomes a
constant tensor, a variable defined in only one branch gets a placeholder on the other side
(the reference's UndefinedVar), identical Python values pass through.  Statements the
conversion cannot express (``break``/``continue`` out of the converted loop, ``return`` not in
tail position, ``global``/``nonlocal``, ``raise``, ``yield``) are left as Python.
"""
import ast
import builtins
import functools
import inspect
import sys
import textwrap
import types

import torch

from ..core.tensor import Tensor, _wrap, _unwrap

_CACHE = {}  # code object -> (converted code object or None, converted source)
_SYSTEM_PREFIXES = ('paddle', 'torch', 'numpy', 'scipy', 'builtins', 'functools', 'collections', 'typing',
                    'abc', 'math', 'copy', 'itertools', 'inspect', 'warnings', 'contextlib', 'einops')


class _Undefined:
    __slots__ = ()

    def __repr__(self):
        return 'UNDEFINED'

    def __bool__(self):
        raise NameError("variable used before assignment (it is only defined in one branch / iteration)")


UNDEFINED = _Undefined()


def _is_static(x):
    t = _unwrap(x)
    return isinstance(t, torch.Tensor) and t.is_meta


def _truth(x):
    return bool(x)


def pack(loc, names):
    """Current values of ``names`` in a frame's ``locals()`` (UNDEFINED when unbound)."""
    return tuple(loc.get(n, UNDEFINED) for n in names)


# ------------------------------------------------------------------ static cond
def _static_cond(pred, true_fn, false_fn, args, names, is_return):
    from ..static.program import default_main_program, Node, Ref, _to_record, _vid_of, _paused
    from ..static.nn import _trace, _meta_like
    prog = default_main_program()
    t_nodes, t_out = _trace(true_fn, args)
    f_nodes, f_out = _trace(false_fn, args)
    t_refs, f_refs, outs = [], [], []

    def as_tensor(v, like=None):
        with _paused():
            if like is not None and (v is UNDEFINED or v is None):
                # placeholder for a variable the branch does not define: never read on that branch,
                # so a scalar suffices (the node output takes the defined side's meta)
                return torch.zeros((), dtype=like.dtype)
            if like is not None:
                return torch.tensor(v, dtype=like.dtype)
            return torch.tensor(v)

    def slot(ta, tb, like=None):
        t_refs.append(_to_record(prog, ta))
        f_refs.append(_to_record(prog, tb))
        m = _meta_like(ta if like is None else like)
        outs.append(prog._new_value(m))
        return _wrap(m)

    def merge(a, b, label):
        if a is b:
            return a
        if (isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)) and type(a) is type(b)
                and len(a) == len(b)):
            items = [merge(x, y, f"{label}[{i}]") for i, (x, y) in enumerate(zip(a, b))]
            return type(a)(*items) if hasattr(a, '_fields') else type(a)(items)
        ta, tb = _unwrap(a), _unwrap(b)
        a_t, b_t = isinstance(ta, torch.Tensor), isinstance(tb, torch.Tensor)
        if a_t and b_t:
            if ta is tb:
                return a
            return slot(ta, tb)
        num = (bool, int, float)
        if a_t and (isinstance(b, num) or b is UNDEFINED or b is None):
            return slot(ta, as_tensor(b, ta), ta)
        if b_t and (isinstance(a, num) or a is UNDEFINED or a is None):
            return slot(as_tensor(a, tb), tb, tb)
        if isinstance(a, num) and isinstance(b, num):
            if a == b and type(a) is type(b):
                return a
            ta = as_tensor(a)
            return slot(ta, as_tensor(b, ta))
        if a is UNDEFINED or b is UNDEFINED:
            return UNDEFINED
        try:
            if a == b:
                return a
        except Exception:  # noqa: BLE001 — objects without a usable __eq__
            pass
        raise ValueError(f"dy2static: '{label}' holds different Python values in the branches of a "
                         f"tensor-dependent if ({a!r} vs {b!r}); make it a Tensor")

    if is_return:
        res = merge(t_out, f_out, 'return value')
    else:
        res = tuple(merge(x, y, n) for x, y, n in zip(t_out, f_out, names))
    prog.nodes.append(Node('cond', None, [Ref(_vid_of(prog, _unwrap(pred)))],
                           {'branches': (t_nodes, t_refs, f_nodes, f_refs)}, outs))
    return res


def convert_ifelse(pred, true_fn, false_fn, args, names, is_return):
    if _is_static(pred):
        return _static_cond(pred, true_fn, false_fn, args, names, is_return)
    return true_fn(*args) if _truth(pred) else false_fn(*args)


def convert_ifexp(pred, true_fn, false_fn):
    if _is_static(pred):
        return _static_cond(pred, lambda: true_fn(), lambda: false_fn(), (), (), True)
    return true_fn() if _truth(pred) else false_fn()


# ------------------------------------------------------------------ static loops
def _to_carried(v, like=None):
    from ..static.program import _paused
    t = _unwrap(v)
    if isinstance(t, torch.Tensor):
        return v if isinstance(v, Tensor) else _wrap(t)
    with _paused():
        return _wrap(torch.tensor(v, dtype=like.dtype) if like is not None else torch.tensor(v))


def _carriable(v):
    return isinstance(_unwrap(v), torch.Tensor) or isinstance(v, (bool, int, float))


def _static_while(cond_fn, body_fn, vals):
    from ..static.nn import while_loop
    vals = list(vals)
    idx = [i for i, v in enumerate(vals) if _carriable(v)]
    init = [_to_carried(vals[i]) for i in idx]

    def full(cv):
        f = list(vals)
        for i, v in zip(idx, cv):
            f[i] = v
        return f

    def c_w(*cv):
        return cond_fn(*full(cv))

    def b_w(*cv):
        out = list(body_fn(*full(cv)))
        return [_to_carried(out[i], _unwrap(c)) for i, c in zip(idx, init)]

    res = while_loop(c_w, b_w, init)
    return tuple(full(res))


def convert_while(cond_fn, body_fn, vals, names):
    from ..static.nn import _trace
    vals = list(vals)
    _, c = _trace(cond_fn, vals)
    if _is_static(c):
        return _static_while(cond_fn, body_fn, vals)
    while _truth(c):
        vals = list(body_fn(*vals))
        c = cond_fn(*vals)
        if _is_static(c):  # the body turned the predicate into a Variable: the rest is a static loop
            return _static_while(cond_fn, body_fn, vals)
    return tuple(vals)


def convert_for_range(rargs, body_fn, vals, names):
    rargs = list(rargs)
    if not any(_is_static(a) for a in rargs):
        r = range(*[int(a) if isinstance(a, Tensor) else a for a in rargs])
        target, rest = vals[0], list(vals[1:])
        for v in r:
            rest = list(body_fn(v, *rest))
            target = v
        return (target, *rest)
    start, stop, step = (0, rargs[0], 1) if len(rargs) == 1 else (rargs[0], rargs[1], rargs[2] if len(rargs) > 2 else 1)
    neg = isinstance(step, (int, float)) and step < 0

    def cond_fn(i, *rest):
        return i > stop if neg else i < stop

    def body(i, *rest):
        out = body_fn(i, *rest)
        return (i + step, *out)

    res = _static_while(cond_fn, body, [start, *vals[1:]])
    return (res[0] - step, *res[1:])


# ------------------------------------------------------------------ logical ops
def convert_logical_and(*fns):
    v = fns[0]()
    for f in fns[1:]:
        if _is_static(v):
            from .. import logical_and
            w = f()
            v = logical_and(v, w if isinstance(w, Tensor) else _to_carried(bool(w)))
            continue
        if not _truth(v):
            return v
        v = f()
    return v


def convert_logical_or(*fns):
    v = fns[0]()
    for f in fns[1:]:
        if _is_static(v):
            from .. import logical_or
            w = f()
            v = logical_or(v, w if isinstance(w, Tensor) else _to_carried(bool(w)))
            continue
        if _truth(v):
            return v
        v = f()
    return v


def convert_logical_not(x):
    if _is_static(x):
        from .. import logical_not
        return logical_not(x)
    return not x


# ------------------------------------------------------------------ calls
def _user_code(obj):
    mod = getattr(obj, '__module__', None) or ''
    return not mod.startswith(_SYSTEM_PREFIXES) and mod != __name__


def convert_call(f):
    """Returns a converted callable for user functions / user Layers reached from converted code."""
    from ..nn.layer.layers import Layer
    if getattr(f, '_jst_not_to_static', False):
        return f
    if isinstance(f, Layer):
        fwd = type(f).forward
        if not _user_code(fwd) or getattr(fwd, '_jst_not_to_static', False) or 'forward' in f.__dict__:
            return f
        conv = convert_function(fwd)
        if conv is fwd:
            return f

        @functools.wraps(f.__call__)
        def call_layer(*a, **k):
            f.__dict__['forward'] = types.MethodType(conv, f)
            try:
                return f(*a, **k)
            finally:
                f.__dict__.pop('forward', None)
        return call_layer
    if isinstance(f, types.MethodType) and isinstance(f.__func__, types.FunctionType) and _user_code(f.__func__):
        return convert_function(f)
    if isinstance(f, types.FunctionType) and _user_code(f):
        return convert_function(f)
    return f


# ------------------------------------------------------------------ AST transform
class _Scan(ast.NodeVisitor):
    """Names a statement list assigns (own scope only) + constructs that block conversion."""

    def __init__(self):
        self.store = []
        self.returns = 0
        self.bad = False        # global/nonlocal/yield/del/raise/await
        self.loop_exit = False  # break/continue that leaves the scanned block
        self._loops = 0

    def _add(self, n):
        if not n.startswith('__jst') and n not in self.store:
            self.store.append(n)

    def visit_Name(self, n):
        if isinstance(n.ctx, ast.Store):
            self._add(n.id)
        elif isinstance(n.ctx, ast.Del):
            self.bad = True

    def _scope(self, n):
        self._add(n.name)

    visit_FunctionDef = visit_AsyncFunctionDef = visit_ClassDef = _scope

    def visit_Lambda(self, n):
        pass

    def visit_ListComp(self, n):
        pass

    visit_SetComp = visit_DictComp = visit_GeneratorExp = visit_ListComp

    def visit_NamedExpr(self, n):
        self._add(n.target.id)
        self.visit(n.value)

    def visit_Return(self, n):
        self.returns += 1
        self.generic_visit(n)

    def _bad(self, n):
        self.bad = True

    visit_Global = visit_Nonlocal = visit_Yield = visit_YieldFrom = visit_Raise = visit_Await = _bad
    visit_Try = visit_With = visit_AsyncWith = visit_AsyncFor = _bad

    def _loop(self, n):
        self._loops += 1
        self.generic_visit(n)
        self._loops -= 1

    visit_For = visit_While = _loop

    def _exit(self, n):
        if self._loops == 0:
            self.loop_exit = True

    visit_Break = visit_Continue = _exit

    def visit_ImportFrom(self, n):
        for a in n.names:
            self._add((a.asname or a.name).split('.')[0])

    visit_Import = visit_ImportFrom


def _scan(stmts):
    s = _Scan()
    for st in stmts:
        s.visit(st)
    return s


def _ends_return(stmts):
    return bool(stmts) and isinstance(stmts[-1], ast.Return)


def _stmt(src):
    return ast.parse(src).body[0]


def _tuple_src(names):
    return '(' + ''.join(f'{n}, ' for n in names) + ')'


class _Fill(ast.NodeTransformer):
    """Replaces placeholder Names ``__JST_k__`` with prepared expressions."""

    def __init__(self, subs):
        self.subs = subs

    def visit_Name(self, n):
        return self.subs.get(n.id, n)


_NO_WRAP_CALLS = {'range', 'len', 'print', 'isinstance', 'issubclass', 'super', 'locals', 'globals', 'type',
                  'getattr', 'setattr', 'hasattr', 'int', 'float', 'bool', 'str', 'list', 'tuple', 'dict', 'set',
                  'zip', 'enumerate', 'map', 'filter', 'min', 'max', 'abs', 'sum', 'any', 'all', 'id', 'repr',
                  'sorted', 'reversed', 'iter', 'next', 'callable', 'vars', 'dir', 'format', 'round', 'divmod'}


class _Dy2St(ast.NodeTransformer):
    def __init__(self):
        self.n = 0
        self.changed = 0

    def _id(self, kind):
        self.n += 1
        return f'__jst_{kind}_{self.n}'

    # ---- blocks
    def _block(self, stmts):
        stmts = list(stmts)
        i = 0
        while i < len(stmts):  # early return: the rest of the block becomes the else branch
            st = stmts[i]
            if isinstance(st, ast.If) and i + 1 < len(stmts):
                if _ends_return(st.body) and not st.orelse:
                    st.orelse = stmts[i + 1:]
                    del stmts[i + 1:]
                elif _ends_return(st.orelse) and not _ends_return(st.body):
                    st.body = st.body + stmts[i + 1:]
                    del stmts[i + 1:]
            i += 1
        out = []
        for st in stmts:
            r = self.visit(st)
            if isinstance(r, list):
                out.extend(r)
            elif r is not None:
                out.append(r)
        return out

    def _mkdef(self, name, params, body, ret):
        fd = _stmt(f"def {name}({', '.join(params)}):\n    pass")
        fd.body = list(body) + ([_stmt(f"return {_tuple_src(ret)}")] if ret is not None else [])
        if not fd.body:
            fd.body = [ast.Pass()]
        return fd

    # ---- scopes
    def visit_FunctionDef(self, node):
        node.body = self._block(node.body)
        return node

    def visit_Lambda(self, node):
        node.body = self.visit(node.body)
        return node

    # ---- expressions
    def visit_BoolOp(self, node):
        self.generic_visit(node)
        fn = 'convert_logical_and' if isinstance(node.op, ast.And) else 'convert_logical_or'
        lambdas = [ast.Lambda(args=ast.arguments(posonlyargs=[], args=[], vararg=None, kwonlyargs=[],
                                                 kw_defaults=[], kwarg=None, defaults=[]), body=v)
                   for v in node.values]
        self.changed += 1
        return ast.copy_location(ast.Call(func=ast.Attribute(value=ast.Name('_jst', ast.Load()), attr=fn,
                                                             ctx=ast.Load()), args=lambdas, keywords=[]), node)

    def visit_UnaryOp(self, node):
        self.generic_visit(node)
        if not isinstance(node.op, ast.Not):
            return node
        self.changed += 1
        return ast.copy_location(ast.Call(func=ast.Attribute(value=ast.Name('_jst', ast.Load()),
                                                             attr='convert_logical_not', ctx=ast.Load()),
                                          args=[node.operand], keywords=[]), node)

    def visit_IfExp(self, node):
        self.generic_visit(node)
        e = _stmt("_jst.convert_ifexp(__JST_0__, lambda: __JST_1__, lambda: __JST_2__)").value
        self.changed += 1
        return ast.copy_location(_Fill({'__JST_0__': node.test, '__JST_1__': node.body,
                                        '__JST_2__': node.orelse}).visit(e), node)

    def visit_Call(self, node):
        self.generic_visit(node)
        f = node.func
        if isinstance(f, ast.Name) and (f.id in _NO_WRAP_CALLS or f.id.startswith('__jst')):
            return node
        if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == '_jst':
            return node
        wrapped = ast.Call(func=ast.Attribute(value=ast.Name('_jst', ast.Load()), attr='convert_call',
                                              ctx=ast.Load()), args=[f], keywords=[])
        node.func = ast.copy_location(wrapped, f)
        self.changed += 1
        return node

    # ---- statements
    def visit_If(self, node):
        node.test = self.visit(node.test)
        node.body = self._block(node.body)
        node.orelse = self._block(node.orelse)
        sb, so = _scan(node.body), _scan(node.orelse)
        if sb.bad or so.bad or sb.loop_exit or so.loop_exit:
            return node
        names = sb.store + [n for n in so.store if n not in sb.store]
        tn, fn_ = self._id('true'), self._id('false')
        sub = {'__JST_0__': node.test}
        if sb.returns or so.returns:
            if not (_ends_return(node.body) and _ends_return(node.orelse) and sb.returns == 1 and so.returns == 1):
                return node
            defs = [self._mkdef(tn, names, node.body, None), self._mkdef(fn_, names, node.orelse, None)]
            call = _stmt(f"return _jst.convert_ifelse(__JST_0__, {tn}, {fn_}, _jst.pack(locals(), "
                         f"{_tuple_src(repr(n) for n in names)}), {_tuple_src(repr(n) for n in names)}, True)")
        else:
            defs = [self._mkdef(tn, names, node.body, names), self._mkdef(fn_, names, node.orelse, names)]
            lhs = f"{_tuple_src(names)} = " if names else ''
            call = _stmt(f"{lhs}_jst.convert_ifelse(__JST_0__, {tn}, {fn_}, _jst.pack(locals(), "
                         f"{_tuple_src(repr(n) for n in names)}), {_tuple_src(repr(n) for n in names)}, False)")
        call = _Fill(sub).visit(call)
        self.changed += 1
        return [ast.copy_location(d, node) for d in defs] + [ast.copy_location(call, node)]

    def visit_While(self, node):
        node.test = self.visit(node.test)
        node.body = self._block(node.body)
        node.orelse = self._block(node.orelse)
        sb = _scan(node.body)
        if node.orelse or sb.bad or sb.loop_exit or sb.returns or not sb.store:
            return node
        names = sb.store
        cn, bn = self._id('cond'), self._id('body')
        cdef = self._mkdef(cn, names, [], None)
        cdef.body = [ast.Return(value=node.test)]
        bdef = self._mkdef(bn, names, node.body, names)
        call = _stmt(f"{_tuple_src(names)} = _jst.convert_while({cn}, {bn}, _jst.pack(locals(), "
                     f"{_tuple_src(repr(n) for n in names)}), {_tuple_src(repr(n) for n in names)})")
        self.changed += 1
        return [ast.copy_location(cdef, node), ast.copy_location(bdef, node), ast.copy_location(call, node)]

    def visit_For(self, node):
        node.iter = self.visit(node.iter)
        node.body = self._block(node.body)
        node.orelse = self._block(node.orelse)
        it = node.iter
        # the iterator may already be wrapped as convert_call(range)(...) — range is in _NO_WRAP_CALLS
        if not (isinstance(node.target, ast.Name) and isinstance(it, ast.Call) and isinstance(it.func, ast.Name)
                and it.func.id == 'range' and not it.keywords and 1 <= len(it.args) <= 3):
            return node
        sb = _scan(node.body)
        if node.orelse or sb.bad or sb.loop_exit or sb.returns:
            return node
        tgt = node.target.id
        names = [n for n in sb.store if n != tgt]
        bn = self._id('for')
        bdef = self._mkdef(bn, [tgt] + names, node.body, names)
        allv = [tgt] + names
        call = _stmt(f"{_tuple_src(allv)} = _jst.convert_for_range(__JST_0__, {bn}, _jst.pack(locals(), "
                     f"{_tuple_src(repr(n) for n in allv)}), {_tuple_src(repr(n) for n in names)})")
        call = _Fill({'__JST_0__': ast.Tuple(elts=list(it.args), ctx=ast.Load())}).visit(call)
        self.changed += 1
        return [ast.copy_location(bdef, node), ast.copy_location(call, node)]


def _convert_code(fn):
    code = fn.__code__
    hit = _CACHE.get(code)
    if hit is not None:
        return hit
    res = (None, '')
    try:
        src = textwrap.dedent(inspect.getsource(fn))
        tree = ast.parse(src)
        fdef = tree.body[0]
        if isinstance(fdef, ast.FunctionDef) and fdef.name == code.co_name:
            fdef.decorator_list = []
            tr = _Dy2St()
            fdef = tr.visit_FunctionDef(fdef)
            if tr.changed:
                ast.increment_lineno(fdef, code.co_firstlineno - 1)
                params = ['_jst'] + [v for v in code.co_freevars if v != '_jst']
                factory = ast.FunctionDef(
                    name='__jst_factory',
                    args=ast.arguments(posonlyargs=[], args=[ast.arg(arg=p) for p in params], vararg=None,
                                       kwonlyargs=[], kw_defaults=[], kwarg=None, defaults=[]),
                    body=[fdef, ast.Return(value=ast.Name(fdef.name, ast.Load()))], decorator_list=[],
                    returns=None, type_comment=None)
                mod = ast.Module(body=[factory], type_ignores=[])
                ast.fix_missing_locations(mod)
                fname = inspect.getsourcefile(fn) or '<dy2static>'
                mcode = compile(mod, fname, 'exec')
                fcode = next(c for c in mcode.co_consts if isinstance(c, types.CodeType))
                inner = next(c for c in fcode.co_consts if isinstance(c, types.CodeType) and c.co_name == fdef.name)
                res = (inner, ast.unparse(fdef))
    except (OSError, TypeError, SyntaxError, StopIteration, IndentationError) as e:  # no source: keep Python
        if _verbose[0]:
            print(f"dy2static: {getattr(fn, '__qualname__', fn)} not converted: {e}", file=sys.stderr)
    _CACHE[code] = res
    return res


_verbose = [0]
_this = sys.modules[__name__]


def convert_function(fn):
    """``fn`` with tensor-dependent control flow converted (``fn`` itself when nothing to convert)."""
    if isinstance(fn, types.MethodType):
        conv = convert_function(fn.__func__)
        return fn if conv is fn.__func__ else types.MethodType(conv, fn.__self__)
    if not isinstance(fn, types.FunctionType) or getattr(fn, '_jst_not_to_static', False):
        return fn
    code, _ = _convert_code(fn)
    if code is None:
        return fn
    cells = dict(zip(fn.__code__.co_freevars, fn.__closure__ or ()))
    closure = tuple(types.CellType(_this) if v == '_jst' else cells[v] for v in code.co_freevars)
    new = types.FunctionType(code, fn.__globals__, fn.__name__, fn.__defaults__, closure)
    new.__kwdefaults__ = fn.__kwdefaults__
    new.__dict__.update(fn.__dict__)
    new.__qualname__, new.__module__, new.__doc__ = fn.__qualname__, fn.__module__, fn.__doc__
    new.__wrapped_dygraph__ = fn
    return new


def converted_source(fn):
    """Source of the converted function (``StaticFunction.code``)."""
    f = fn.__func__ if isinstance(fn, types.MethodType) else fn
    if not isinstance(f, types.FunctionType):
        return ''
    code, src = _convert_code(f)
    if code is None:
        try:
            return textwrap.dedent(inspect.getsource(f))
        except (OSError, TypeError):
            return ''
    return src


__all__ = ['convert_function', 'convert_call', 'convert_ifelse', 'convert_while', 'convert_for_range',
           'convert_logical_and', 'convert_logical_or', 'convert_logical_not', 'convert_ifexp', 'UNDEFINED',
           'converted_source']
del builtins
