"""This framework's own opcode translator — the SOT front end (reference: python/paddle/jit/sot/
opcode_translator/: an executor that simulates a function's CPython bytecode, records the tensor
work into a static program, breaks the graph where it has to run Python, and guards each
translation on what it was built for).

Model.  ``OpcodeTranslator(fn)(*args)`` interprets ``fn``'s bytecode (CPython 3.10) itself:

* A **region** starts at the function entry and right after every graph break.  It is translated
  by interpreting the instructions *symbolically*: every tensor in the frame state (locals, the
  value stack, own cell variables) is replaced by a data Variable of a fresh static ``Program``,
  so every tensor operation the instructions reach — paddle APIs, Layers, Tensor methods and
  operators, user functions inlined instruction by instruction — is recorded by the static
  recorder (static/program.py), while plain Python (shape arithmetic, containers, branches on
  Python values, unrolled loops) is evaluated once and baked into the region under its guards.
* A region ends at the first instruction that needs concrete values or has an effect outside the
  region: a branch on a tensor, ``float()/int()/bool()/.numpy()/.item()/.tolist()`` of a tensor,
  ``print``, f-strings of tensors, a store into an object / container / global that existed before
  the region, a mutating method of such a container, an exception, or an opcode this translator
  does not model.  That instruction runs concretely (on the region's real outputs) and the next
  region starts after it.
* A translated region is kept with its **guards**: the start state's structure (tensor shapes,
  dtypes and stop_gradient, Python values, object identities, Layer training flags), the globals /
  closure cells it read, and the simple attribute values it read from pre-existing objects.  A
  later call whose state satisfies them runs the region's Program on the Executor (hand-written
  GEMM substitutions, IR fusion passes on the GPU, autograd kept) and rebuilds the end state from
  the region's template — the Python inside the region is not re-run; anything else re-translates.

``with`` blocks are entered and exited concretely (graph breaks at SETUP_WITH and at the block's
end), so the region inside runs under the context (grad mode and AMP state are part of every
region's guard); an exception closes the open blocks and propagates.  Functions with generators or
try / except handlers run eagerly (no translation); a call into such a function from a region is a
graph break.  Translation never changes results:
whatever cannot be modelled runs as plain Python.
"""
import builtins
import dis
import inspect
import operator
import types

import torch

from ..core.tensor import Tensor, _wrap

_STATS = {'regions': 0, 'recorded': 0, 'hits': 0, 'runs': 0, 'breaks': 0, 'eager_calls': 0, 'nodes': 0}

_BINARY = {
    'BINARY_ADD': operator.add, 'BINARY_SUBTRACT': operator.sub, 'BINARY_MULTIPLY': operator.mul,
    'BINARY_TRUE_DIVIDE': operator.truediv, 'BINARY_FLOOR_DIVIDE': operator.floordiv, 'BINARY_MODULO': operator.mod,
    'BINARY_POWER': operator.pow, 'BINARY_MATRIX_MULTIPLY': operator.matmul, 'BINARY_SUBSCR': operator.getitem,
    'BINARY_AND': operator.and_, 'BINARY_OR': operator.or_, 'BINARY_XOR': operator.xor,
    'BINARY_LSHIFT': operator.lshift, 'BINARY_RSHIFT': operator.rshift,
    'INPLACE_ADD': operator.iadd, 'INPLACE_SUBTRACT': operator.isub, 'INPLACE_MULTIPLY': operator.imul,
    'INPLACE_TRUE_DIVIDE': operator.itruediv, 'INPLACE_FLOOR_DIVIDE': operator.ifloordiv,
    'INPLACE_MODULO': operator.imod, 'INPLACE_POWER': operator.ipow, 'INPLACE_MATRIX_MULTIPLY': operator.imatmul,
    'INPLACE_AND': operator.iand, 'INPLACE_OR': operator.ior, 'INPLACE_XOR': operator.ixor,
    'INPLACE_LSHIFT': operator.ilshift, 'INPLACE_RSHIFT': operator.irshift,
}
_UNARY = {'UNARY_NEGATIVE': operator.neg, 'UNARY_POSITIVE': operator.pos, 'UNARY_NOT': operator.not_,
          'UNARY_INVERT': operator.invert}
_COMPARE = {'<': operator.lt, '<=': operator.le, '==': operator.eq, '!=': operator.ne, '>': operator.gt,
            '>=': operator.ge}
_SUPPORTED = set(_BINARY) | set(_UNARY) | {
    'NOP', 'POP_TOP', 'ROT_TWO', 'ROT_THREE', 'ROT_FOUR', 'ROT_N', 'DUP_TOP', 'DUP_TOP_TWO',
    'LOAD_CONST', 'LOAD_FAST', 'STORE_FAST', 'DELETE_FAST', 'LOAD_GLOBAL', 'STORE_GLOBAL', 'LOAD_DEREF',
    'STORE_DEREF', 'LOAD_CLOSURE', 'LOAD_ATTR', 'STORE_ATTR', 'DELETE_ATTR', 'LOAD_METHOD', 'CALL_METHOD',
    'CALL_FUNCTION', 'CALL_FUNCTION_KW', 'CALL_FUNCTION_EX', 'STORE_SUBSCR', 'DELETE_SUBSCR', 'COMPARE_OP',
    'IS_OP', 'CONTAINS_OP', 'BUILD_TUPLE', 'BUILD_LIST', 'BUILD_SET', 'BUILD_MAP', 'BUILD_CONST_KEY_MAP',
    'BUILD_SLICE', 'BUILD_STRING', 'FORMAT_VALUE', 'LIST_APPEND', 'SET_ADD', 'MAP_ADD', 'LIST_EXTEND',
    'SET_UPDATE', 'LIST_TO_TUPLE', 'DICT_MERGE', 'DICT_UPDATE', 'UNPACK_SEQUENCE', 'UNPACK_EX', 'GET_ITER',
    'FOR_ITER', 'JUMP_FORWARD', 'JUMP_ABSOLUTE', 'POP_JUMP_IF_FALSE', 'POP_JUMP_IF_TRUE', 'JUMP_IF_FALSE_OR_POP',
    'JUMP_IF_TRUE_OR_POP', 'RETURN_VALUE', 'MAKE_FUNCTION', 'EXTENDED_ARG', 'GET_LEN', 'IMPORT_NAME',
    'IMPORT_FROM', 'SETUP_WITH', 'POP_BLOCK', 'WITH_EXCEPT_START', 'RERAISE', 'POP_EXCEPT',
}
_NO_TRANSLATE_FLAGS = inspect.CO_GENERATOR | inspect.CO_COROUTINE | inspect.CO_ASYNC_GENERATOR | \
    inspect.CO_ITERABLE_COROUTINE
_BREAK_CALLS = {builtins.print, builtins.input, builtins.open, builtins.breakpoint, builtins.exec, builtins.eval}
_VALUE_CALLS = {builtins.float, builtins.int, builtins.bool, builtins.complex, builtins.str, builtins.repr,
                builtins.format, builtins.hash}
_TENSOR_VALUE_METHODS = {'numpy', 'item', 'tolist', '__bool__', '__float__', '__int__', '__index__', '__array__',
                         '__repr__', '__str__', '__format__', 'cpu_numpy'}
_CONTEXT_METHODS = {'__enter__', '__exit__'}  # context-manager entry / exit: run concretely
_MUTATORS = {'append', 'extend', 'insert', 'pop', 'remove', 'clear', 'update', 'setdefault', 'add', 'discard',
             'popitem', 'sort', 'reverse', '__setitem__', '__delitem__', 'set_value', 'copy_', 'fill_'}
_LIBS = ('paddle', 'torch', 'numpy', 'builtins', 'functools', 'typing', 'collections', 'math', 'operator',
         'abc', 'contextlib', 'inspect', 'itertools', 'copy', 'warnings', 'einops', 'scipy', 'enum', 'dataclasses')
_SIMPLE = (bool, int, float, str, type(None), complex, bytes)


class _Break(Exception):
    """The current instruction must run concretely: the region ends before it."""


class _Code:
    """A decoded code object: instructions, offset -> index, whether this translator models it."""
    _cache = {}

    def __init__(self, code):
        self.code = code
        self.instrs = [i for i in dis.get_instructions(code)]
        self.index = {ins.offset: k for k, ins in enumerate(self.instrs)}
        self.ok = not (code.co_flags & _NO_TRANSLATE_FLAGS) and all(i.opname in _SUPPORTED for i in self.instrs)
        # try / finally handlers are not modelled; a POP_BLOCK then only closes a `with` block
        self.ok = self.ok and not any(i.opname == 'SETUP_FINALLY' for i in self.instrs)

    @classmethod
    def of(cls, code):
        c = cls._cache.get(code)
        if c is None:
            c = cls._cache[code] = cls(code)
        return c


def _is_sym(v):
    return isinstance(v, Tensor) and v._t.is_meta


def _any_sym(obj, depth=0):
    if _is_sym(obj):
        return True
    if depth > 3:
        return False
    if isinstance(obj, (list, tuple)):
        return any(_any_sym(o, depth + 1) for o in obj)
    if isinstance(obj, dict):
        return any(_any_sym(o, depth + 1) for o in obj.values())
    return False


def _user_function(f):
    mod = getattr(f, '__module__', None) or ''
    return isinstance(f, types.FunctionType) and mod.split('.')[0] not in _LIBS


class _Frame:
    def __init__(self, fn, args, kwargs):
        self.fn = fn
        self.dc = _Code.of(fn.__code__)
        self.globals = fn.__globals__
        b = self.globals.get('__builtins__', builtins)
        self.builtins = b if isinstance(b, dict) else b.__dict__
        code = fn.__code__
        pos = code.co_varnames[:code.co_argcount]
        if any(n.startswith('.') for n in pos):  # comprehension bodies: implicit '.0' iterator argument
            self.locals = dict(zip(pos, args))
        else:
            # the code object's own parameters (not a functools.wraps target's signature)
            bound = inspect.signature(fn, follow_wrapped=False).bind(*args, **kwargs)
            bound.apply_defaults()
            self.locals = dict(bound.arguments)
        self.cells = {}
        for name in code.co_cellvars:
            cell = types.CellType()
            if name in self.locals:
                cell.cell_contents = self.locals.pop(name)
            self.cells[name] = cell
        self.own_cells = tuple(code.co_cellvars)
        for name, cell in zip(code.co_freevars, fn.__closure__ or ()):
            self.cells[name] = cell
        self.stack = []
        self.pc = 0
        self.withs = []  # exit methods of the active `with` blocks (entered concretely)


class _Ctx:
    """Translation context of one region (symbolic) or None for concrete execution."""

    def __init__(self):
        self.created = set()
        self.keep = []           # objects whose ids are in `created` (ids stay unique)
        self.guards = []         # callables: True while the region's assumptions hold
        self.depth = 0
        self.local_vals = {}     # start-state Python locals the region read: name -> value
        self.assigned = set()    # top-frame locals the region stored before reading
        self.top = None          # the region's own frame (locals guards apply to it only)

    def mark(self, obj):
        self.created.add(id(obj))
        self.keep.append(obj)
        return obj

    def outer(self, obj):
        return id(obj) not in self.created


# ---------------------------------------------------------------------------------- interpreter
def _call(ctx, fn, args, kwargs):
    if ctx is None:
        return fn(*args, **kwargs)
    sym = _any_sym(args) or _any_sym(kwargs)
    self_obj = getattr(fn, '__self__', None)
    if fn in _BREAK_CALLS:
        raise _Break('side effect')
    if fn in _VALUE_CALLS and sym:
        raise _Break('tensor value')
    name = getattr(fn, '__name__', '')
    if name in _CONTEXT_METHODS:
        raise _Break('context manager entry / exit')
    if _is_sym(self_obj) and name in _TENSOR_VALUE_METHODS:
        raise _Break('tensor value')
    if name in _MUTATORS and self_obj is not None and not isinstance(self_obj, types.ModuleType) and \
            ctx.outer(self_obj) and not _is_sym(self_obj):
        raise _Break('mutation of a pre-existing object')
    if fn is builtins.super and not args:
        raise _Break('zero-argument super')  # handled by the caller frame
    if fn is not getattr:  # a library call may read a pre-existing container's elements
        for a_ in list(args) + list(kwargs.values()):
            _guard_contents(ctx, a_)
        if self_obj is not None and not isinstance(self_obj, types.ModuleType) and name not in _MUTATORS:
            _guard_contents(ctx, self_obj)
    # user Python: inlined instruction by instruction (its breaks become a break at this call)
    f, pre = fn, ()
    if isinstance(fn, types.MethodType) and isinstance(fn.__func__, types.FunctionType):
        f, pre = fn.__func__, (fn.__self__,)
    else:
        from ..nn.layer.layers import Layer
        if isinstance(fn, Layer) and 'forward' not in fn.__dict__:
            fwd = type(fn).forward
            if _user_function(fwd) and not _layer_hooks(fn):
                f, pre = fwd, (fn,)
    if _user_function(f) and _Code.of(f.__code__).ok and ctx.depth < 16:
        ctx.depth += 1
        try:
            return _run_frame(_Frame(f, pre + tuple(args), kwargs), ctx)
        finally:
            ctx.depth -= 1
    try:
        return fn(*args, **kwargs)
    except _Break:
        raise
    except Exception as e:  # noqa: BLE001 — whatever the symbolic values cannot do runs concretely
        raise _Break(f'{type(e).__name__}: {e}') from e


def _layer_hooks(layer):
    d = layer.__dict__
    return bool(d.get('_forward_pre_hooks') or d.get('_forward_post_hooks'))


def _run_frame(fr, ctx):
    """Interpret ``fr`` from its pc to RETURN_VALUE (nested symbolic frames)."""
    while True:
        r = _step(fr, ctx)
        if r is not None:
            return r[1]


def _step(fr, ctx):
    """Execute the instruction at fr.pc; returns ('return', value) at RETURN_VALUE, else None.
    In symbolic mode raises _Break BEFORE changing any state."""
    ins = fr.dc.instrs[fr.pc]
    op, arg, st = ins.opname, ins.argval, fr.stack
    nxt = fr.pc + 1

    def jump(offset):
        fr.pc = fr.dc.index[offset]

    if op in _BINARY:
        a, b = st[-2], st[-1]
        if op == 'BINARY_SUBSCR':
            _guard_contents(ctx, a)
        if ctx is not None and op == 'BINARY_SUBSCR' and not _is_sym(a) and not isinstance(a, (list, tuple, dict)) \
                and not hasattr(a, '__getitem__'):
            raise _Break('subscript')
        if ctx is not None and op.startswith('INPLACE') and ctx.outer(a) and isinstance(a, (list, dict, set)):
            raise _Break('in-place update of a pre-existing container')
        v = _call(ctx, _BINARY[op], (a, b), {})
        if ctx is not None and op == 'BINARY_SUBSCR' and ctx.outer(a) and isinstance(v, _SIMPLE) and not _is_sym(a):
            ctx.guards.append(lambda a=a, b=b, v=v: _safe_eq(lambda: a[b], v))
        del st[-2:]
        st.append(v)
    elif op in _UNARY:
        a = st[-1]
        if ctx is not None and op == 'UNARY_NOT' and _is_sym(a):
            raise _Break('truth value of a tensor')
        st[-1] = _call(ctx, _UNARY[op], (a,), {})
    elif op == 'NOP' or op == 'EXTENDED_ARG':
        pass
    elif op == 'POP_TOP':
        st.pop()
    elif op == 'ROT_TWO':
        st[-1], st[-2] = st[-2], st[-1]
    elif op == 'ROT_THREE':
        st[-1], st[-2], st[-3] = st[-2], st[-3], st[-1]
    elif op == 'ROT_FOUR':
        st[-1], st[-2], st[-3], st[-4] = st[-2], st[-3], st[-4], st[-1]
    elif op == 'ROT_N':
        st.insert(len(st) - ins.arg + 1, st.pop())
    elif op == 'DUP_TOP':
        st.append(st[-1])
    elif op == 'DUP_TOP_TWO':
        st.extend(st[-2:])
    elif op == 'LOAD_CONST':
        st.append(arg)
    elif op == 'LOAD_FAST':
        if arg not in fr.locals:
            raise UnboundLocalError(arg)
        v = fr.locals[arg]
        if ctx is not None and fr is ctx.top and arg not in ctx.assigned and isinstance(v, _SIMPLE):
            ctx.local_vals.setdefault(arg, v)  # keyed by type only: the value it read is a guard
        st.append(v)
    elif op == 'STORE_FAST':
        if ctx is not None and fr is ctx.top:
            ctx.assigned.add(arg)
        fr.locals[arg] = st.pop()
    elif op == 'DELETE_FAST':
        del fr.locals[arg]
    elif op == 'LOAD_GLOBAL':
        if arg in fr.globals:
            v = fr.globals[arg]
            g = fr.globals
            if ctx is not None:
                ctx.guards.append(lambda g=g, n=arg, v=v: g.get(n, _MISSING) is v)
        else:
            v = fr.builtins[arg]
        st.append(v)
    elif op == 'STORE_GLOBAL':
        if ctx is not None:
            raise _Break('global store')
        fr.globals[arg] = st.pop()
    elif op == 'LOAD_CLOSURE':
        st.append(fr.cells[arg])
    elif op == 'LOAD_DEREF':
        cell = fr.cells[arg]
        v = cell.cell_contents
        if ctx is not None and arg not in fr.own_cells:
            ctx.guards.append(lambda c=cell, v=v: _cell_is(c, v))
        st.append(v)
    elif op == 'STORE_DEREF':
        if ctx is not None and arg not in fr.own_cells:
            raise _Break('closure store')
        fr.cells[arg].cell_contents = st.pop()
    elif op == 'LOAD_ATTR':
        obj = st[-1]
        v = _call(ctx, getattr, (obj, arg), {}) if ctx is not None else getattr(obj, arg)
        if ctx is not None and ctx.outer(obj) and not _is_sym(obj) and not isinstance(obj, (types.ModuleType, type)) \
                and not isinstance(v, (types.MethodType, types.BuiltinMethodType)):
            if isinstance(v, _SIMPLE):  # a value the translation may have branched on
                ctx.guards.append(lambda o=obj, n=arg, v=v: _safe_eq(lambda: getattr(o, n), v))
            else:  # an object (sublayer, parameter, buffer) the region captured: the same one
                ctx.guards.append(lambda o=obj, n=arg, v=v: _attr_is(o, n, v))
        st[-1] = v
    elif op == 'STORE_ATTR':
        obj = st[-1]
        if ctx is not None and ctx.outer(obj):
            raise _Break('attribute store on a pre-existing object')
        setattr(obj, arg, st[-2])
        del st[-2:]
    elif op == 'DELETE_ATTR':
        if ctx is not None and ctx.outer(st[-1]):
            raise _Break('attribute delete')
        delattr(st.pop(), arg)
    elif op == 'STORE_SUBSCR':
        obj = st[-2]
        if ctx is not None and (ctx.outer(obj) or _is_sym(obj)):
            raise _Break('item store on a pre-existing object')
        obj[st[-1]] = st[-3]
        del st[-3:]
    elif op == 'DELETE_SUBSCR':
        if ctx is not None and ctx.outer(st[-2]):
            raise _Break('item delete')
        del st[-2][st[-1]]
        del st[-2:]
    elif op == 'LOAD_METHOD':
        obj = st[-1]
        m = _call(ctx, getattr, (obj, arg), {}) if ctx is not None else getattr(obj, arg)
        st[-1] = m  # bound method (the NULL / self slot pair of CPython collapsed into one value)
        st.append(_NOSELF)
    elif op == 'CALL_METHOD':
        n = ins.arg
        args = tuple(st[len(st) - n:])
        fn = st[-n - 2]
        v = _call_any(fr, ctx, fn, args, {})
        del st[len(st) - n - 2:]
        st.append(v)
    elif op == 'CALL_FUNCTION':
        n = ins.arg
        args = tuple(st[len(st) - n:])
        fn = st[-n - 1]
        v = _call_any(fr, ctx, fn, args, {})
        del st[len(st) - n - 1:]
        st.append(v)
    elif op == 'CALL_FUNCTION_KW':
        names = st[-1]
        n = ins.arg
        vals = st[len(st) - n - 1:-1]
        nk = len(names)
        args = tuple(vals[:n - nk])
        kwargs = dict(zip(names, vals[n - nk:]))
        fn = st[-n - 2]
        v = _call_any(fr, ctx, fn, args, kwargs)
        del st[len(st) - n - 2:]
        st.append(v)
    elif op == 'CALL_FUNCTION_EX':
        has_kw = ins.arg & 1
        kwargs = dict(st[-1]) if has_kw else {}
        args = tuple(st[-1 - has_kw])
        fn = st[-2 - has_kw]
        v = _call_any(fr, ctx, fn, args, kwargs)
        del st[len(st) - 2 - has_kw:]
        st.append(v)
    elif op == 'COMPARE_OP':
        v = _call(ctx, _COMPARE[arg], (st[-2], st[-1]), {})
        del st[-2:]
        st.append(v)
    elif op == 'IS_OP':
        v = (st[-2] is st[-1]) != bool(ins.arg)
        del st[-2:]
        st.append(v)
    elif op == 'CONTAINS_OP':
        if ctx is not None and (_is_sym(st[-1]) or _is_sym(st[-2])):
            raise _Break('membership test on a tensor')
        _guard_contents(ctx, st[-1])
        v = (st[-2] in st[-1]) != bool(ins.arg)
        del st[-2:]
        st.append(v)
    elif op in ('BUILD_TUPLE', 'BUILD_LIST', 'BUILD_SET'):
        n = ins.arg
        items = st[len(st) - n:] if n else []
        v = tuple(items) if op == 'BUILD_TUPLE' else (list(items) if op == 'BUILD_LIST' else set(items))
        if n:
            del st[len(st) - n:]
        st.append(ctx.mark(v) if ctx is not None and op != 'BUILD_TUPLE' else v)
    elif op == 'BUILD_MAP':
        n = ins.arg
        items = st[len(st) - 2 * n:] if n else []
        v = {items[2 * i]: items[2 * i + 1] for i in range(n)}
        if n:
            del st[len(st) - 2 * n:]
        st.append(ctx.mark(v) if ctx is not None else v)
    elif op == 'BUILD_CONST_KEY_MAP':
        n = ins.arg
        keys = st[-1]
        v = dict(zip(keys, st[len(st) - n - 1:-1]))
        del st[len(st) - n - 1:]
        st.append(ctx.mark(v) if ctx is not None else v)
    elif op == 'BUILD_SLICE':
        n = ins.arg
        v = slice(*st[len(st) - n:])
        del st[len(st) - n:]
        st.append(v)
    elif op == 'BUILD_STRING':
        n = ins.arg
        v = ''.join(st[len(st) - n:]) if n else ''
        if n:
            del st[len(st) - n:]
        st.append(v)
    elif op == 'FORMAT_VALUE':
        has_spec = (ins.arg & 0x04) == 0x04
        spec = st[-1] if has_spec else ''
        val = st[-1 - has_spec]
        if ctx is not None and _any_sym(val):
            raise _Break('formatting a tensor')
        conv = ins.arg & 0x03
        if conv == 1:
            val = str(val)
        elif conv == 2:
            val = repr(val)
        elif conv == 3:
            val = ascii(val)
        v = format(val, spec)
        del st[len(st) - 1 - has_spec:]
        st.append(v)
    elif op == 'LIST_APPEND':
        lst = st[-1 - ins.arg]
        if ctx is not None and ctx.outer(lst):
            raise _Break('append to a pre-existing list')
        lst.append(st.pop())
    elif op == 'SET_ADD':
        st[-1 - ins.arg].add(st.pop())
    elif op == 'MAP_ADD':
        d = st[-2 - ins.arg]
        d[st[-2]] = st[-1]
        del st[-2:]
    elif op in ('LIST_EXTEND', 'SET_UPDATE', 'DICT_MERGE', 'DICT_UPDATE'):
        tgt = st[-1 - ins.arg]
        if ctx is not None and ctx.outer(tgt):
            raise _Break('update of a pre-existing container')
        src = st[-1]
        if op == 'LIST_EXTEND':
            tgt.extend(src)
        elif op == 'SET_UPDATE':
            tgt.update(src)
        else:
            if op == 'DICT_MERGE' and set(tgt) & set(src):
                raise TypeError('got multiple values for keyword argument')
            tgt.update(src)
        st.pop()
    elif op == 'LIST_TO_TUPLE':
        st[-1] = tuple(st[-1])
    elif op == 'UNPACK_SEQUENCE':
        seq = st[-1]
        _guard_contents(ctx, seq)
        items = list(_call(ctx, list, (seq,), {})) if ctx is not None else list(seq)
        if len(items) != ins.arg:
            raise ValueError(f"expected {ins.arg} values to unpack, got {len(items)}")
        st.pop()
        st.extend(reversed(items))
    elif op == 'UNPACK_EX':
        seq = list(_call(ctx, list, (st[-1],), {})) if ctx is not None else list(st[-1])
        before, after = ins.arg & 0xFF, ins.arg >> 8
        mid = seq[before:len(seq) - after if after else len(seq)]
        st.pop()
        vals = seq[:before] + [ctx.mark(mid) if ctx is not None else mid] + (seq[len(seq) - after:] if after else [])
        st.extend(reversed(vals))
    elif op == 'GET_ITER':
        obj = st[-1]
        _guard_contents(ctx, obj)
        it = _call(ctx, iter, (obj,), {}) if ctx is not None else iter(obj)
        st[-1] = ctx.mark(it) if ctx is not None else it
    elif op == 'GET_LEN':
        st.append(_call(ctx, len, (st[-1],), {}) if ctx is not None else len(st[-1]))
    elif op == 'FOR_ITER':
        it = st[-1]
        if ctx is not None and ctx.outer(it):
            raise _Break('iteration of a pre-existing iterator')
        try:
            v = next(it)
        except StopIteration:
            st.pop()
            jump(arg)
            return None
        st.append(v)
    elif op in ('JUMP_FORWARD', 'JUMP_ABSOLUTE'):
        jump(arg)
        return None
    elif op in ('POP_JUMP_IF_FALSE', 'POP_JUMP_IF_TRUE'):
        c = st[-1]
        if ctx is not None and _any_sym(c):
            raise _Break('branch on a tensor')
        t = _truth(ctx, c)
        st.pop()
        if t == (op == 'POP_JUMP_IF_TRUE'):
            jump(arg)
            return None
    elif op in ('JUMP_IF_FALSE_OR_POP', 'JUMP_IF_TRUE_OR_POP'):
        c = st[-1]
        if ctx is not None and _any_sym(c):
            raise _Break('branch on a tensor')
        t = _truth(ctx, c)
        if t == (op == 'JUMP_IF_TRUE_OR_POP'):
            jump(arg)
            return None
        st.pop()
    elif op == 'RETURN_VALUE':
        return ('return', st.pop())
    elif op == 'SETUP_WITH':  # runs concretely: __enter__ is a side effect of the call
        if ctx is not None:
            raise _Break('with-block entry')
        cm = st.pop()
        exit_fn = type(cm).__exit__.__get__(cm)
        res = type(cm).__enter__(cm)
        st.append(exit_fn)
        fr.withs.append(exit_fn)
        st.append(res)
    elif op == 'POP_BLOCK':  # closes a `with` block (its exit call follows); concrete
        if ctx is not None:
            raise _Break('with-block exit')
        fr.withs.pop()
    elif op in ('WITH_EXCEPT_START', 'RERAISE', 'POP_EXCEPT'):  # exception paths: never reached
        raise RuntimeError(f'opcode translator: {op} outside an exception')
    elif op == 'IMPORT_NAME':  # function-level import (idempotent; the module is baked into a region)
        mod = __import__(arg, fr.globals, None, st[-1], st[-2])
        del st[-2:]
        st.append(mod)
    elif op == 'IMPORT_FROM':
        try:
            st.append(getattr(st[-1], arg))
        except AttributeError:
            import importlib
            st.append(importlib.import_module(st[-1].__name__ + '.' + arg))
    elif op == 'MAKE_FUNCTION':
        flags = ins.arg
        qual, code = st[-1], st[-2]
        k = len(st) - 2
        closure = annotations = kwdefaults = defaults = None
        if flags & 0x08:
            k -= 1
            closure = st[k]
        if flags & 0x04:
            k -= 1
            annotations = st[k]
        if flags & 0x02:
            k -= 1
            kwdefaults = st[k]
        if flags & 0x01:
            k -= 1
            defaults = st[k]
        f = types.FunctionType(code, fr.globals, qual.rsplit('.', 1)[-1], defaults, closure)
        f.__qualname__ = qual
        if kwdefaults:
            f.__kwdefaults__ = kwdefaults
        if annotations:
            f.__annotations__ = dict(zip(annotations[::2], annotations[1::2])) \
                if isinstance(annotations, tuple) else annotations
        del st[k:]
        st.append(ctx.mark(f) if ctx is not None else f)
    else:  # pragma: no cover — _Code.ok excludes it
        raise NotImplementedError(op)
    fr.pc = nxt
    return None


class _NoSelf:
    __slots__ = ()


_NOSELF = _NoSelf()
_MISSING = object()


def _call_any(fr, ctx, fn, args, kwargs):
    if args and args[-1] is _NOSELF:  # LOAD_METHOD's placeholder (the method is already bound)
        args = args[:-1]
    if fn is builtins.super and not args:  # zero-argument super(): __class__ cell + first argument
        cls = fr.cells['__class__'].cell_contents
        first = fr.fn.__code__.co_varnames[0]
        obj = fr.locals[first] if first in fr.locals else fr.cells[first].cell_contents
        return super(cls, obj)
    return _call(ctx, fn, args, kwargs)


def _truth(ctx, c):
    if ctx is None:
        return bool(c)
    if isinstance(c, _SIMPLE + (list, tuple, dict, set)) or c is None:
        return bool(c)
    try:
        return bool(c)
    except Exception as e:  # noqa: BLE001
        raise _Break('truth value') from e


def _same(a, b):
    return type(a) is type(b) and a == b


def _safe_eq(get, v):
    try:
        return get() == v
    except Exception:  # noqa: BLE001
        return False


def _attr_is(o, n, v):
    try:
        return getattr(o, n) is v
    except Exception:  # noqa: BLE001
        return False


def _cell_is(cell, v):
    try:
        return cell.cell_contents is v
    except ValueError:
        return False


# --------------------------------------------------------------------------------- frame state
def _state_key(fr):
    """Hashable description of the frame state a region depends on: the structure of locals,
    stack and own cells; tensors by (shape, dtype, stop_gradient, device); Python values by
    value; other objects by identity (Layers with their training flags)."""
    from ..core import amp_dispatch as _disp
    a = _disp.STATE
    parts = [fr.pc, torch.is_grad_enabled(), (a.active, a.level, a.dtype, a.white, a.black, a.use_promote),
             len(fr.withs)]
    for name in sorted(fr.locals):
        v = fr.locals[name]
        # Python scalars in locals by type: the values a region reads become its local guards
        parts.append((name, ('V', type(v)) if isinstance(v, _SIMPLE) else _vkey(v)))
    parts.append(('|stack',) + tuple(_vkey(v) for v in fr.stack))
    for name in fr.own_cells:
        c = fr.cells[name]
        try:
            parts.append(('cell', name, _vkey(c.cell_contents)))
        except ValueError:
            parts.append(('cell', name, 'empty'))
    return tuple(parts)


def _contents(v, depth=0):
    """Full value key of a container (elements by value) for content guards."""
    if isinstance(v, (list, tuple)) and depth < 6:
        return (type(v).__name__,) + tuple(_contents(x, depth + 1) for x in v)
    if isinstance(v, dict) and depth < 6:
        return ('dict',) + tuple((k, _contents(x, depth + 1)) for k, x in v.items())
    if isinstance(v, _SIMPLE):
        return ('V', type(v), v)
    return _vkey(v, depth)


def _guard_contents(ctx, obj):
    """A region read the elements of a pre-existing list / dict / set: it replays only while they
    are the same."""
    if ctx is not None and type(obj) in (list, dict, set) and ctx.outer(obj):
        snap = _contents(list(obj) if type(obj) is set else obj)
        ctx.guards.append(lambda o=obj, k=snap: _contents(list(o) if type(o) is set else o) == k)


def _vkey(v, depth=0):
    if isinstance(v, Tensor):
        t = v._t
        return ('T', tuple(t.shape), t.dtype, t.requires_grad, t.device.type)
    if isinstance(v, torch.Tensor):
        return ('t', id(v))
    if isinstance(v, _SIMPLE):
        return ('V', type(v), v)
    # tuples by value; lists / dicts by shape only — their Python contents are guarded where a
    # region reads them (_guard_contents), and a list a region passes through is handed back by slot
    if depth < 4 and type(v) is tuple:
        return ('tuple',) + tuple(_vkey(x, depth + 1) for x in v)
    if depth < 4 and type(v) is list:
        return ('list',) + tuple((k, _vkey(x, depth + 1)) for k, x in enumerate(v) if isinstance(x, Tensor))
    if depth < 4 and type(v) is dict:
        return ('dict',) + tuple((k, _vkey(x, depth + 1) if isinstance(x, (Tensor, list, tuple, dict)) else
                                  (('V', type(x)) if isinstance(x, _SIMPLE) else _vkey(x, depth + 1)))
                                 for k, x in v.items() if isinstance(k, _SIMPLE))
    from ..nn.layer.layers import Layer
    if isinstance(v, Layer):
        return ('L', id(v), tuple(m.training for m in v.sublayers(include_self=True)))
    if v is _NOSELF:
        return ('noself',)
    if isinstance(v, types.MethodType) and v.__name__ == '__exit__':  # an open `with` block's exit
        return ('exit', type(v.__self__))
    if isinstance(v, (types.MethodType, types.BuiltinMethodType)) and getattr(v, '__self__', None) is not None \
            and not isinstance(v.__self__, types.ModuleType):  # a bound method: its object, its name
        return ('M', id(v.__self__), v.__name__)
    if hasattr(type(v), '__exit__') and hasattr(type(v), '__enter__'):  # a context manager object
        return ('cm', type(v))
    return ('O', id(v))


class _Slots:
    """Tensors of a frame state in a fixed walk order (feeds of a region)."""

    @staticmethod
    def collect(fr):
        out = []

        def walk(v, depth=0):
            if isinstance(v, Tensor):
                out.append(v)
            elif depth < 4 and type(v) in (tuple, list):
                for x in v:
                    walk(x, depth + 1)
            elif depth < 4 and type(v) is dict:
                for x in v.values():
                    walk(x, depth + 1)
        for name in sorted(fr.locals):
            walk(fr.locals[name])
        for v in fr.stack:
            walk(v)
        for name in fr.own_cells:
            try:
                walk(fr.cells[name].cell_contents)
            except ValueError:
                pass
        return out


def _replace(v, mapping, ctx, depth=0):
    """The symbolic image of a start-state value (tensors -> their data Variables)."""
    if isinstance(v, Tensor) and id(v) in mapping:
        return mapping[id(v)]
    if depth < 4 and type(v) is tuple:
        return tuple(_replace(x, mapping, ctx, depth + 1) for x in v)
    if depth < 4 and type(v) is list and any(isinstance(x, Tensor) for x in v):
        return [_replace(x, mapping, ctx, depth + 1) for x in v]  # a copy: still a pre-existing object
    if depth < 4 and type(v) is dict and any(isinstance(x, Tensor) for x in v.values()):
        return {k: _replace(x, mapping, ctx, depth + 1) for k, x in v.items()}
    return v


class _Region:
    """One translated region: Program, feeds (walk order of the start state's tensors), the end
    state template, the end pc (or a return), the guards."""

    def __init__(self):
        self.prog = None
        self.feed_names = []
        self.end_pc = None
        self.returned = False
        self.tpl_locals = None
        self.tpl_stack = None
        self.tpl_cells = None
        self.tpl_ret = None
        self.guards = []
        self.out_vids = ()
        self.reason = None
        self.local_vals = {}


def _template(v, prog, inputs, depth=0, origin=None):
    """End-state value -> template: ('in', k) an input tensor, ('out', vid) a recorded value,
    ('slot', path) a start-state object handed through (the replaying call's own object),
    ('tup'/'list'/'dict', ...) containers (rebuilt per replay), ('c', v) a baked value."""
    if origin is not None and not isinstance(v, _SIMPLE + (Tensor,)) and id(v) in origin:
        return ('slot', origin[id(v)])
    if isinstance(v, Tensor):
        if id(v) in inputs:
            return ('in', inputs[id(v)])
        if v._t.is_meta:
            vid = prog._val.get(id(v._t))
            if vid is None:
                raise _Break('a tensor the recorder did not produce')
            return ('out', vid)
        return ('c', v)
    if isinstance(v, (types.MethodType, types.BuiltinMethodType)) and \
            getattr(v, '__self__', None) is not None and not isinstance(v.__self__, types.ModuleType):
        # a bound method (LOAD_METHOD's value left on the stack at a break): bound afresh to the
        # replaying call's object — the recording's object may be the region's private copy
        ts = _template(v.__self__, prog, inputs, depth + 1, origin)
        if ts[0] in ('slot', 'in', 'out'):  # an identity the replay reproduces (a rebuilt container would not)
            return ('meth', ts, v.__name__)
    if type(v) in _ITER_TYPES:  # a list / tuple / range iterator: its source and position
        red = v.__reduce__()
        if len(red) >= 2 and red[0] is builtins.iter and len(red[1]) == 1:
            return ('iter', _template(red[1][0], prog, inputs, depth + 1, origin), red[2] if len(red) > 2 else 0)
    if depth < 6 and type(v) is tuple:
        return ('tup', [_template(x, prog, inputs, depth + 1, origin) for x in v])
    if depth < 6 and type(v) is list:
        return ('list', [_template(x, prog, inputs, depth + 1, origin) for x in v])
    if depth < 6 and type(v) is dict:
        return ('dict', [(k, _template(x, prog, inputs, depth + 1, origin)) for k, x in v.items()])
    return ('c', v)


_ITER_TYPES = (type(iter([])), type(iter(())), type(iter(range(0))), type(iter(range(1 << 70))))
# objects the region may create and hand on baked into its template: immutable, so a replay can
# share them (anything else created by the region — e.g. a closure over the region's symbolic
# values — makes the region untranslatable: it would leak recording-time state into every replay)
_SHAREABLE = _SIMPLE + (range, slice, type, types.ModuleType, types.BuiltinFunctionType, frozenset)


def _baked_unsafe(t, ctx):
    kind = t[0]
    if kind == 'c':
        v = t[1]
        return id(v) in ctx.created and not isinstance(v, _SHAREABLE) and not isinstance(v, Tensor)
    if kind in ('tup', 'list'):
        return any(_baked_unsafe(x, ctx) for x in t[1])
    if kind == 'dict':
        return any(_baked_unsafe(x, ctx) for _, x in t[1])
    if kind in ('iter', 'meth'):
        return _baked_unsafe(t[1], ctx)
    return False


def _slot_value(start, path):
    kind, key = path
    return start[kind][key]


def _materialize(t, env, feeds, start=None):
    kind = t[0]
    if kind == 'slot':
        return _slot_value(start, t[1])
    if kind == 'in':
        return feeds[t[1]]
    if kind == 'out':
        return _wrap(env[t[1]])
    if kind == 'tup':
        return tuple(_materialize(x, env, feeds, start) for x in t[1])
    if kind == 'list':
        return [_materialize(x, env, feeds, start) for x in t[1]]
    if kind == 'dict':
        return {k: _materialize(x, env, feeds, start) for k, x in t[1]}
    if kind == 'meth':
        return getattr(_materialize(t[1], env, feeds, start), t[2])
    if kind == 'iter':
        it = iter(_materialize(t[1], env, feeds, start))
        if t[2]:
            it.__setstate__(t[2])
        return it
    return t[1]


def _out_vids(t, acc):
    kind = t[0]
    if kind == 'out':
        acc.add(t[1])
    elif kind in ('tup', 'list'):
        for x in t[1]:
            _out_vids(x, acc)
    elif kind == 'dict':
        for _, x in t[1]:
            _out_vids(x, acc)
    elif kind in ('iter', 'meth'):
        _out_vids(t[1], acc)
    return acc


_PD_DT = {torch.float32: 'float32', torch.float16: 'float16', torch.bfloat16: 'bfloat16', torch.float64: 'float64',
          torch.int64: 'int64', torch.int32: 'int32', torch.bool: 'bool', torch.int8: 'int8', torch.uint8: 'uint8',
          torch.int16: 'int16', torch.complex64: 'complex64', torch.complex128: 'complex128'}


def _translate(fr):
    """Translate the region starting at fr.pc (the frame itself is not modified)."""
    from ..static.program import Program, program_guard, data, _start_recording, _stop_recording, _recorder
    reg = _Region()
    tensors = _Slots.collect(fr)
    if any(t._t.dtype not in _PD_DT for t in tensors):
        return None
    prog = Program()
    sfr = _Frame.__new__(_Frame)
    sfr.__dict__.update(fr.__dict__)
    ctx = _Ctx()
    ctx.top = sfr
    started = _recorder[0] is None
    if started:
        _start_recording()
    try:
        with program_guard(prog):
            mapping, names, inputs = {}, [], {}
            for k, t in enumerate(tensors):
                if id(t) in mapping:
                    continue
                nm = f'sot_in{k}'
                v = data(nm, list(t._t.shape), _PD_DT[t._t.dtype])
                v.stop_gradient = not t._t.requires_grad
                mapping[id(t)] = v
                names.append(nm)
                inputs[id(v)] = len(names) - 1
            sfr.locals = {n: _replace(v, mapping, ctx) for n, v in fr.locals.items()}
            sfr.stack = [_replace(v, mapping, ctx) for v in fr.stack]
            cells = dict(fr.cells)
            for name in fr.own_cells:
                c = types.CellType()
                try:
                    c.cell_contents = _replace(fr.cells[name].cell_contents, mapping, ctx)
                except ValueError:
                    pass
                cells[name] = c
            sfr.cells = cells
            origin = {}
            for n_, v_ in sfr.locals.items():
                origin.setdefault(id(v_), ('L', n_))
            for k_, v_ in enumerate(sfr.stack):
                origin.setdefault(id(v_), ('S', k_))
            for n_ in fr.own_cells:
                try:
                    origin.setdefault(id(cells[n_].cell_contents), ('C', n_))
                except ValueError:
                    pass
            start = sfr.pc
            while True:
                pc0 = sfr.pc
                try:
                    r = _step(sfr, ctx)
                except _Break as e:
                    reg.reason = str(e)
                    sfr.pc = pc0
                    break
                if r is not None:
                    reg.returned = True
                    reg.tpl_ret = _template(r[1], prog, inputs, origin=origin)
                    break
            if not reg.returned and sfr.pc == start and not prog.nodes:
                return None  # breaks at once: nothing to translate
            reg.end_pc = sfr.pc
            if not reg.returned:
                reg.tpl_locals = {n: _template(v, prog, inputs, origin=origin) for n, v in sfr.locals.items()}
                reg.tpl_stack = [_template(v, prog, inputs, origin=origin) for v in sfr.stack]
                reg.tpl_cells = {}
                for name in fr.own_cells:
                    try:
                        reg.tpl_cells[name] = _template(sfr.cells[name].cell_contents, prog, inputs, origin=origin)
                    except ValueError:
                        pass
    except _Break:
        return None
    finally:
        if started:
            _stop_recording()
    ends = [reg.tpl_ret] if reg.returned else list(reg.tpl_locals.values()) + reg.tpl_stack + \
        list(reg.tpl_cells.values())
    if any(_baked_unsafe(t, ctx) for t in ends):
        return None
    acc = set()
    for t in ([reg.tpl_ret] if reg.returned else list(reg.tpl_locals.values()) + reg.tpl_stack +
              list(reg.tpl_cells.values())):
        _out_vids(t, acc)
    reg.out_vids = tuple(sorted(acc))
    reg.prog, reg.feed_names, reg.guards = prog, names, ctx.guards
    reg.local_vals = dict(ctx.local_vals)
    _STATS['regions'] += 1
    _STATS['recorded'] += 1 if prog.nodes else 0
    _STATS['nodes'] += len(prog.nodes)
    if reg.reason is not None:
        _STATS['breaks'] += 1
    return reg


def _run_region(fr, reg):
    """Run a translated region on fr's real state; returns ('return', value) or None (fr advanced)."""
    from ..static.executor import run_program
    from ..core.place import current_device
    tensors = _Slots.collect(fr)
    uniq, seen = [], set()
    for t in tensors:
        if id(t) not in seen:
            seen.add(id(t))
            uniq.append(t)
    feeds = uniq
    _STATS['runs'] += 1
    if reg.prog.nodes:
        dev = feeds[0]._t.device if feeds else current_device()
        env = run_program(reg.prog, dict(zip(reg.feed_names, [t._t for t in feeds])), dev,
                          grad=torch.is_grad_enabled(), fetch=reg.out_vids)
    else:
        env = {}
    start = {'L': dict(fr.locals), 'S': list(fr.stack), 'C': {}}
    for name in fr.own_cells:
        try:
            start['C'][name] = fr.cells[name].cell_contents
        except ValueError:
            pass
    if reg.returned:
        return ('return', _materialize(reg.tpl_ret, env, feeds, start))
    fr.locals = {n: _materialize(t, env, feeds, start) for n, t in reg.tpl_locals.items()}
    fr.stack = [_materialize(t, env, feeds, start) for t in reg.tpl_stack]
    for name, t in reg.tpl_cells.items():
        fr.cells[name].cell_contents = _materialize(t, env, feeds, start)
    fr.pc = reg.end_pc
    return None


class OpcodeTranslator:
    """``fn`` (a function or bound method) run through this translator; see the module doc."""

    def __init__(self, fn):
        self.self_obj = None
        if not isinstance(fn, (types.FunctionType, types.MethodType)) and callable(fn) and \
                isinstance(getattr(type(fn), '__call__', None), types.FunctionType):
            fn = types.MethodType(type(fn).__call__, fn)  # a callable object (a Layer): its __call__
        if isinstance(fn, types.MethodType):
            self.self_obj, fn = fn.__self__, fn.__func__
        self.fn = fn
        self.ok = isinstance(fn, types.FunctionType) and _Code.of(fn.__code__).ok
        self.cache = {}  # state key -> [regions]
        self.neg = set()  # pcs whose instruction always breaks at once

    def __call__(self, *args, **kwargs):
        if not self.ok:
            _STATS['eager_calls'] += 1
            return self.fn(*((self.self_obj,) + args if self.self_obj is not None else args), **kwargs)
        full = ((self.self_obj,) + args) if self.self_obj is not None else args
        fr = _Frame(self.fn, full, kwargs)
        try:
            return self._run(fr)
        except BaseException as e:
            # exceptions are not modelled inside the frame: close its open `with` blocks the way
            # CPython's handler would (innermost first) and propagate
            while fr.withs:
                fr.withs.pop()(type(e), e, e.__traceback__)
            raise

    def _run(self, fr):
        while True:
            reg = None
            if fr.pc not in self.neg:
                key = _state_key(fr)
                for r in self.cache.get(key, ()):
                    if all(_same(fr.locals.get(n, _MISSING), v) for n, v in r.local_vals.items()) and \
                            all(g() for g in r.guards):
                        reg = r
                        _STATS['hits'] += 1
                        break
                if reg is None:
                    reg = _translate(fr)
                    if reg is not None:
                        self.cache.setdefault(key, []).append(reg)
                    else:
                        self.neg.add(fr.pc)  # breaks at its first instruction: run it concretely
            if reg is not None:
                res = _run_region(fr, reg)
                if res is not None:
                    return res[1]
            # the break instruction, concretely
            r = _step(fr, None)
            if r is not None:
                return r[1]


def stats():
    return dict(_STATS)


__all__ = ['OpcodeTranslator', 'stats']
