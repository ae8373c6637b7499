"""paddle.pir — the program-IR namespace of the reference's 3.x static graph (python/paddle/pir/).

This framework records static programs as an op list over torch functions (static/program.py);
``paddle.pir`` exposes it under the reference names: ``Program`` (the static Program), ``Value`` /
``OpResult`` (a program variable), ``Operation`` views of the recorded ops (``name()``,
``operands()``, ``results()``), ``translate_to_pir`` (identity: programs are already in this IR),
and ``save`` / ``load`` of the reference's PIR JSON file format (static/pir_json.py; reference
paddle/fluid/pir/serialize_deserialize, python/paddle/static/pir_io.py:527/610)."""
from .static.program import Program, Ref, Const  # noqa: F401
from .core.tensor import Tensor as Value  # noqa: F401

OpResult = Value


class Operation:
    """A read-only view of one recorded op of a Program."""

    def __init__(self, prog, node):
        self._prog, self._node = prog, node

    def name(self):
        t = self._node.target
        n = getattr(t, '__name__', None) or type(t).__name__
        return n if '.' in n else 'pd_op.' + n

    def operands(self):
        def walk(a, out):
            if isinstance(a, (Ref, Const)):
                out.append(a)
            elif isinstance(a, (list, tuple)):
                for x in a:
                    walk(x, out)
            elif isinstance(a, dict):
                for x in a.values():
                    walk(x, out)
            return out
        return walk(list(self._node.args) + [self._node.kwargs], [])

    def results(self):
        o = self._node.outs
        return [o] if isinstance(o, int) else list(o or [])

    num_operands = property(lambda self: len(self.operands()))
    num_results = property(lambda self: len(self.results()))

    def __repr__(self):
        return f"<Operation {self.name()} operands={len(self.operands())} results={len(self.results())}>"


def ops_of(program):
    """Operations of a Program's global block, in program order."""
    return [Operation(program, n) for n in program.nodes]


def translate_to_pir(program_desc):
    """Programs are recorded directly in this framework's IR: returns its argument."""
    return program_desc


def is_fake_value(value):
    return False


def save(program, path, feed_vars, fetch_vars):
    """``<path>.json`` (+ ``.pdiparams``) in the reference's PIR serialization format."""
    from .static.io import save_pir
    if not save_pir(feed_vars, fetch_vars, path, program):
        raise NotImplementedError("program uses an operator outside the PIR-exportable set")


def load(path):
    """A PIR ``.json`` program (and ``.pdiparams`` if present) as an executable Program."""
    import os
    from .static.pir_json import load as _load
    from .static.pdmodel import load_params
    from .core.place import current_device
    with open(path if path.endswith('.json') else path + '.json', 'rb') as f:
        prog = _load(f.read())
    prefix = path[:-5] if path.endswith('.json') else path
    if os.path.exists(prefix + '.pdiparams'):
        with open(prefix + '.pdiparams', 'rb') as f:
            load_params(prog, f.read(), current_device())
    return prog
