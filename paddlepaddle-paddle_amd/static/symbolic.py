"""Symbolic dimensions of static Programs (reference: paddle/pir/include/dialect/shape/utils/dim_expr.h
DimExpr, shape_analysis.h ShapeConstraintIRAnalysis).

A dynamic dim of a fed Variable (``None`` / -1) is a symbol ``S<i>`` (i = the dim position, so the
batch dims of two feeds are one symbol and the executor checks that the feeds agree).  Meta tensors
still need concrete extents for torch's shape inference, so a symbol's *carrier* extent is a large
prime (``program.SENTINELS``); what the user's Python code sees, however, is a ``SymInt``: an
``int`` whose value is the carrier extent and which carries its ``DimExpr``.  Arithmetic on
SymInts (+ - * // %, and with plain ints) builds the expression as it computes the value, so shape
arithmetic such as ``x.shape[0] * x.shape[1]`` or ``math.prod(x.shape)`` reaches a recorded op as
the expression ``S0*S1``; the Executor evaluates it with the fed extents.

Where Python drops the subclass through ``int(s)`` / ``operator.index(s)`` (``range``, slicing),
the conversion itself is recorded: the recording program's *value table* maps each value that
escaped that way to its expression, and only those plain ints are re-specialised.  An unrelated
constant that merely happens to be a multiple of a carrier extent is left alone (the old
prime-factoring rule re-specialised any such multiple).  Conversions that bypass both hooks
(numpy reductions over a shape) are not seen: keep shape arithmetic in Python ints.

Extents of op outputs are decoded by unique factorisation over the carrier primes (an extent of a
meta tensor that is c * S0^a * S1^b ... can only have come from symbolic extents: torch's shape
inference multiplies / divides them), which is how shapes computed inside torch — views,
reshapes, matmuls — turn back into expressions when Python reads them.
"""
import operator

_OPS = {'+': operator.add, '-': operator.sub, '*': operator.mul, '//': operator.floordiv, '%': operator.mod,
        'max': max, 'min': min}


class DimExpr:
    __slots__ = ()

    def eval(self, env):
        raise NotImplementedError

    def symbols(self):
        return set()


class Sym(DimExpr):
    """Symbol S<i>: the dynamic extent at dim position i of the feeds."""
    __slots__ = ('i',)

    def __init__(self, i):
        self.i = i

    def eval(self, env):
        return env[self.i]

    def symbols(self):
        return {self.i}

    def __repr__(self):
        return f"S{self.i}"

    def to_json(self):
        return ['s', self.i]


class Lit(DimExpr):
    __slots__ = ('v',)

    def __init__(self, v):
        self.v = int(v)

    def eval(self, env):
        return self.v

    def __repr__(self):
        return str(self.v)

    def to_json(self):
        return self.v


class Bin(DimExpr):
    __slots__ = ('op', 'a', 'b')

    def __init__(self, op, a, b):
        self.op, self.a, self.b = op, a, b

    def eval(self, env):
        return _OPS[self.op](self.a.eval(env), self.b.eval(env))

    def symbols(self):
        return self.a.symbols() | self.b.symbols()

    def __repr__(self):
        if self.op in ('max', 'min'):
            return f"{self.op}({self.a!r}, {self.b!r})"
        return f"({self.a!r}{self.op}{self.b!r})"

    def to_json(self):
        return [self.op, self.a.to_json(), self.b.to_json()]


class Neg(DimExpr):
    __slots__ = ('a',)

    def __init__(self, a):
        self.a = a

    def eval(self, env):
        return -self.a.eval(env)

    def symbols(self):
        return self.a.symbols()

    def __repr__(self):
        return f"-{self.a!r}"

    def to_json(self):
        return ['neg', self.a.to_json()]


def expr_from_json(j):
    if isinstance(j, int):
        return Lit(j)
    if j[0] == 's':
        return Sym(j[1])
    if j[0] == 'neg':
        return Neg(expr_from_json(j[1]))
    return Bin(j[0], expr_from_json(j[1]), expr_from_json(j[2]))


# ---------------------------------------------------------------------------------- SymInt
_TABLE = [None]   # value table of the program being recorded (dict value -> DimExpr), or None
_GETTER = [None]  # static/program.py: the recording program's value table (None when not recording)


def _note(v, e):
    t = _TABLE[0]
    if t is None and _GETTER[0] is not None:
        t = _GETTER[0]()
    if t is not None and not isinstance(e, Lit):
        t.setdefault(v, e)


def _ex(x):
    return x.expr if isinstance(x, SymInt) else Lit(int.__int__(x))


def _mk(v, e):
    if isinstance(e, Lit) or not e.symbols():
        return int(v)
    return SymInt(v, e)


def _binop(op, rev=False):
    f = _OPS[op]

    def method(self, other):
        if isinstance(other, bool) or not isinstance(other, int):
            return NotImplemented
        a, b = (other, self) if rev else (self, other)
        v = f(int.__int__(a), int.__int__(b))
        return _mk(v, Bin(op, _ex(a), _ex(b)))
    return method


class SymInt(int):
    """An int (the carrier extent) that carries its symbolic DimExpr."""

    def __new__(cls, value, expr):
        o = int.__new__(cls, value)
        o.expr = expr
        return o

    def __int__(self):
        _note(int.__int__(self), self.expr)  # the plain int escapes: remember what it stands for
        return int.__int__(self)

    __add__ = _binop('+')
    __radd__ = _binop('+', True)
    __sub__ = _binop('-')
    __rsub__ = _binop('-', True)
    __mul__ = _binop('*')
    __rmul__ = _binop('*', True)
    __floordiv__ = _binop('//')
    __rfloordiv__ = _binop('//', True)
    __mod__ = _binop('%')
    __rmod__ = _binop('%', True)

    def __neg__(self):
        return _mk(-int.__int__(self), Neg(self.expr))

    def __pos__(self):
        return self

    def __abs__(self):
        return self if int.__int__(self) >= 0 else -self

    def __index__(self):
        _note(int.__index__(self), self.expr)
        return int.__index__(self)

    def __repr__(self):
        return int.__repr__(self)

    def __reduce__(self):
        return (int, (int.__int__(self),))

    def __deepcopy__(self, memo):
        return self

    def __copy__(self):
        return self


def sym_max(a, b):
    """max() that keeps the expression (Python's max returns one operand unchanged)."""
    v = max(int.__int__(a), int.__int__(b))
    return _mk(v, Bin('max', _ex(a), _ex(b)))


def sym_min(a, b):
    v = min(int.__int__(a), int.__int__(b))
    return _mk(v, Bin('min', _ex(a), _ex(b)))


def decode_extent(v, sentinels):
    """The DimExpr of a carrier-valued extent (c * prod S_i^k), or None when no carrier divides it."""
    v = int.__int__(v)
    if v <= 0:
        return None
    rest, e = v, None
    for i, s in enumerate(sentinels):
        while rest % s == 0:
            rest //= s
            e = Sym(i) if e is None else Bin('*', e, Sym(i))
    if e is None:
        return None
    return e if rest == 1 else Bin('*', Lit(rest), e)


def symbolize(v, sentinels):
    """v as a SymInt when it is a carrier-valued extent, else unchanged."""
    if isinstance(v, SymInt) or isinstance(v, bool) or not isinstance(v, int):
        return v
    e = decode_extent(v, sentinels)
    return v if e is None else SymInt(v, e)


class recording_table:
    """Context: SymInts created inside note their values in ``table`` (a program's value table)."""

    def __init__(self, table):
        self.table = table

    def __enter__(self):
        self.prev = _TABLE[0]
        _TABLE[0] = self.table

    def __exit__(self, *a):
        _TABLE[0] = self.prev
