"""Program decomposition (reference: python/paddle/decomposition/decomp.py ``decompose`` ->
core.sinking_decomp).

Walks the recorded op list of a static ``Program`` (``static/program.py``) and replaces every op that
has a registered composite rule (``rules.py``), is allowed by the white/black lists and lies in
``[start_index, end_index)`` by the primitive ops its rule records.  The rule is traced on the
node's meta values under the program recorder, so the replacement nodes are ordinary program nodes
(the Executor, ``jit.save`` and the ProgramDesc exporter see primitives).  The decomposed op's output
values keep their ids, so every later consumer and the caller's ``src_vars`` stay valid; as in the
reference, ``decompose`` returns the (possibly replaced) ``src_vars``.
"""
import torch

from ..static import program as P
from . import rules  # noqa: F401  (registers the built-in rules)
from .register import get_decomp_rule

# recorded torch callable name -> reference operator name
_OP_NAMES = {
    'softmax': 'pd_op.softmax', 'log_softmax': 'pd_op.log_softmax', 'gelu': 'pd_op.gelu', 'silu': 'pd_op.silu',
    'relu': 'pd_op.relu', 'relu6': 'pd_op.relu6', 'leaky_relu': 'pd_op.leaky_relu', 'elu': 'pd_op.elu',
    'hardsigmoid': 'pd_op.hardsigmoid', 'hardswish': 'pd_op.hardswish', 'layer_norm': 'pd_op.layer_norm',
    'rms_norm': 'pd_op.rms_norm', 'mean': 'pd_op.mean', 'addmm': 'pd_op.addmm', 'linear': 'pd_op.linear',
    'batch_norm': 'pd_op.batch_norm', 'group_norm': 'pd_op.group_norm', 'dropout': 'pd_op.dropout',
    'square': 'pd_op.square', 'reciprocal': 'pd_op.reciprocal', 'flatten': 'pd_op.flatten',
    'squeeze': 'pd_op.squeeze', 'unsqueeze': 'pd_op.unsqueeze', 'stack': 'pd_op.stack',
    'embedding': 'pd_op.embedding', 'clamp': 'pd_op.clip', 'clip': 'pd_op.clip',
}

# the reference's prim_config["forward_blacklist"] analogue (ops never decomposed by default)
_prim_config = {'forward_blacklist': set(), 'prim_enabled': False}


def op_name(node):
    """Reference operator name of a recorded node ('' when it has none)."""
    if node.kind != 'torch':
        return ''
    return _OP_NAMES.get(getattr(node.target, '__name__', ''), '')


def _vid_meta(prog):
    out = {}
    for t in prog._keep:
        v = prog._val.get(id(t))
        if v is not None:
            out[v] = t
    return out


def _materialise(prog, obj, vmeta, forced):
    if isinstance(obj, P.Ref):
        return vmeta[obj.vid]
    if isinstance(obj, P.Const):
        t = prog.consts[obj.cid]
        forced.add(id(t))
        return t
    if isinstance(obj, tuple) and hasattr(obj, '_fields'):
        return type(obj)(*[_materialise(prog, o, vmeta, forced) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_materialise(prog, o, vmeta, forced) for o in obj)
    if isinstance(obj, dict):
        return {k: _materialise(prog, v, vmeta, forced) for k, v in obj.items()}
    return obj


def _rename(obj, old, new):
    if isinstance(obj, P.Ref):
        return P.Ref(new) if obj.vid == old else obj
    if isinstance(obj, tuple) and hasattr(obj, '_fields'):
        return type(obj)(*[_rename(o, old, new) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_rename(o, old, new) for o in obj)
    if isinstance(obj, dict):
        return {k: _rename(v, old, new) for k, v in obj.items()}
    return obj


def _rename_outs(outs, old, new):
    if isinstance(outs, list):
        return [_rename_outs(o, old, new) for o in outs]
    return new if outs == old else outs


def _flat_outs(outs):
    if isinstance(outs, list):
        r = []
        for o in outs:
            r.extend(_flat_outs(o))
        return r
    return [] if outs is None else [outs]


def _flat_tensors(obj):
    if isinstance(obj, torch.Tensor):
        return [obj]
    if isinstance(obj, (list, tuple)):
        r = []
        for o in obj:
            r.extend(_flat_tensors(o))
        return r
    return []


def _decompose_node(prog, node, rule, vmeta):
    forced = set()
    args = _materialise(prog, node.args, vmeta, forced)
    kwargs = _materialise(prog, node.kwargs, vmeta, forced)
    saved, prog.nodes = prog.nodes, []
    prog._force_record_ids = forced
    started = P._recorder[0] is None
    if started:
        P._start_recording()
    try:
        with P.program_guard(prog):
            res = rule(*args, **kwargs)
    finally:
        if started:
            P._stop_recording()
        prog._force_record_ids = None
        new_nodes, prog.nodes = prog.nodes, saved
    old_outs = _flat_outs(node.outs)
    new_ts = _flat_tensors(res)
    if len(old_outs) != len(new_ts):
        raise RuntimeError(f"decomposition rule of {op_name(node)} returned {len(new_ts)} outputs, "
                           f"the op has {len(old_outs)}")
    for old_vid, t in zip(old_outs, new_ts):
        ref_meta = vmeta.get(old_vid)
        if ref_meta is not None and (list(t.shape) != list(ref_meta.shape) or t.dtype != ref_meta.dtype):
            raise RuntimeError(f"decomposition rule of {op_name(node)}: output {list(t.shape)} {t.dtype} does not "
                               f"match the op's {list(ref_meta.shape)} {ref_meta.dtype}")
        new_vid = prog._val.get(id(t))
        producer = None
        if new_vid is not None:
            for nn in new_nodes:
                if new_vid in _flat_outs(nn.outs):
                    producer = nn
        if producer is None:  # the rule returned one of its inputs (identity): alias node
            src = new_vid if new_vid is not None else None
            if src is None:
                raise RuntimeError(f"decomposition rule of {op_name(node)} returned a value outside the program")
            new_nodes.append(P.Node('torch', torch.Tensor.view_as, [P.Ref(src), P.Ref(src)], {}, old_vid))
            continue
        producer.outs = _rename_outs(producer.outs, new_vid, old_vid)
        for nn in new_nodes:
            nn.args = _rename(nn.args, new_vid, old_vid)
            nn.kwargs = _rename(nn.kwargs, new_vid, old_vid)
    return new_nodes


def decompose(program, src_vars, blacklist=frozenset(), whitelist=frozenset(), start_index=0, end_index=-1):
    """Replace the ops of ``program`` that have a composite rule by primitive ops.

    The decomposed set is (ops in [start_index, end_index) with a rule, restricted to ``whitelist``
    when it is non-empty) minus ``blacklist`` (which wins over the whitelist).  Names are the
    reference operator names ('pd_op.softmax').  Returns ``src_vars`` (their values keep their ids).
    """
    assert isinstance(start_index, int) and isinstance(end_index, int)
    blacklist = set(_prim_config['forward_blacklist']) | set(blacklist)
    whitelist = set(whitelist)
    nodes = program.nodes
    end = len(nodes) if end_index == -1 else min(end_index, len(nodes))
    vmeta = _vid_meta(program)
    out = []
    for i, node in enumerate(nodes):
        name = op_name(node) if start_index <= i < end else ''
        rule = get_decomp_rule(name) if name else None
        if rule is None or name in blacklist or (whitelist and name not in whitelist):
            out.append(node)
            continue
        try:
            repl = _decompose_node(program, node, rule, vmeta)
        except NotImplementedError:
            out.append(node)  # this instance is outside the rule (e.g. training-mode batch_norm)
            continue
        vmeta = _vid_meta(program)
        out.extend(repl)
    program.nodes = out
    return src_vars
