"""Program serialisation + inference-model IO (reference: python/paddle/static/io.py
save_inference_model / load_inference_model / serialize_program / save / load;
python/paddle/jit/api.py:908 jit.save reuses the same format).

Format (ours, not the reference protobuf):
* ``<prefix>.pdmodel``  — JSON: feeds (name, value id, shape with -1, dtype), fetch value ids,
  and the op list.  Targets are named (``Tensor.reshape``, ``torch._C._nn.linear``,
  ``Tensor.@T`` for properties); loading resolves names only inside ``torch`` / ``paddle.ops``
  namespaces — nothing from the file is executed as code.
* ``<prefix>.pdiparams`` — safetensors with every captured constant (parameters, buffers).
"""
from ..framework.flags import pa_flag  # noqa: E402
import importlib
import json
import os

import torch

from ..core.tensor import Tensor, _wrap
from . import symbolic as _sym
from .program import Program, Node, Ref, Const, default_main_program, _vid_of, _paused

_NAMESPACES = ('torch', 'torch.nn.functional', 'torch._C._nn', 'torch.linalg', 'torch.special', 'torch.fft',
               'torch._C._linalg', 'torch._C._special', 'torch._C._fft', 'torch._C._VariableFunctions')
_DTYPES = {str(d).replace('torch.', ''): d for d in (
    torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int8, torch.int16, torch.int32, torch.int64,
    torch.uint8, torch.bool, torch.complex64, torch.complex128, torch.float8_e4m3fn, torch.float8_e5m2)}


# ----------------------------------------------------------------- target names
def target_name(f):
    name = getattr(f, '__name__', None)
    if name == '__get__' and type(getattr(f, '__self__', None)).__name__ == 'getset_descriptor':
        return 'Tensor.@' + f.__self__.__name__
    if name and (getattr(torch.Tensor, name, None) is f or getattr(torch._C.TensorBase, name, None) is f):
        return 'Tensor.' + name
    mod = getattr(f, '__module__', None)
    if mod and (mod == 'torch' or mod.startswith('torch.') or mod.startswith('paddle.ops')):
        try:
            if getattr(importlib.import_module(mod), name, None) is f:
                return f"{mod}:{name}"
        except ImportError:
            pass
    for ns in _NAMESPACES:
        try:
            m = importlib.import_module(ns) if not ns.startswith('torch._C.') else _cmod(ns)
        except ImportError:
            continue
        if m is not None and getattr(m, name, None) is f:
            return f"{ns}:{name}"
    raise ValueError(f"cannot serialise op target {f!r}")


def _cmod(ns):
    obj = torch._C
    for part in ns.split('.')[2:]:
        obj = getattr(obj, part, None)
        if obj is None:
            return None
    return obj


def resolve_target(s):
    if s.startswith('Tensor.@'):
        desc = torch._C.TensorBase.__dict__.get(s[8:]) or torch.Tensor.__dict__.get(s[8:])
        if desc is None:
            raise ValueError(f"unknown tensor property {s}")
        return desc.__get__
    if s.startswith('Tensor.'):
        return getattr(torch.Tensor, s[7:])
    mod, name = s.split(':')
    if not (mod == 'torch' or mod.startswith('torch.') or mod.startswith('paddle.ops')):
        raise ValueError(f"op namespace {mod} is not allowed in a serialised program")
    m = _cmod(mod) if mod.startswith('torch._C.') else importlib.import_module(mod)
    return getattr(m, name)


# ----------------------------------------------------------------- value encoding
def _enc(v):
    if isinstance(v, Ref):
        return {'r': v.vid}
    if isinstance(v, Const):
        return {'c': v.cid}
    if isinstance(v, _sym.SymInt):  # a dynamic-dim expression (static/symbolic.py)
        return {'sym': [int(v), v.expr.to_json()]}
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, torch.dtype):
        return {'dt': str(v).replace('torch.', '')}
    if isinstance(v, torch.device):
        return {'dev': v.type}
    if isinstance(v, torch.Size):
        return {'sz': list(v)}
    if isinstance(v, slice):
        return {'sl': [_enc(v.start), _enc(v.stop), _enc(v.step)]}
    if v is Ellipsis:
        return {'el': 1}
    if isinstance(v, torch.memory_format):
        return {'mf': str(v).replace('torch.', '')}
    if isinstance(v, torch.layout):
        return {'ly': str(v).replace('torch.', '')}
    if isinstance(v, list):
        return {'l': [_enc(x) for x in v]}
    if isinstance(v, tuple):
        return {'t': [_enc(x) for x in v]}
    if isinstance(v, dict):
        return {'d': {k: _enc(x) for k, x in v.items()}}
    raise ValueError(f"cannot serialise op argument {v!r}")


def _dec(v):
    if not isinstance(v, dict):
        return v
    if 'r' in v:
        return Ref(v['r'])
    if 'c' in v:
        return Const(v['c'])
    if 'sym' in v:
        return _sym.SymInt(v['sym'][0], _sym.expr_from_json(v['sym'][1]))
    if 'dt' in v:
        return _DTYPES[v['dt']]
    if 'dev' in v:
        return torch.device(v['dev'])
    if 'sz' in v:
        return torch.Size(v['sz'])
    if 'sl' in v:
        return slice(*[_dec(x) for x in v['sl']])
    if 'el' in v:
        return Ellipsis
    if 'mf' in v:
        return getattr(torch, v['mf'])
    if 'ly' in v:
        return getattr(torch, v['ly'])
    if 'l' in v:
        return [_dec(x) for x in v['l']]
    if 't' in v:
        return tuple(_dec(x) for x in v['t'])
    if 'd' in v:
        return {k: _dec(x) for k, x in v['d'].items()}
    raise ValueError(f"bad encoded value {v}")


def _enc_nodes(nodes):
    out = []
    for n in nodes:
        if n.kind in ('minimize', 'backward', 'grad'):
            continue
        if n.kind == 'checkpoint':  # a recompute segment: its ops, inline (recompute is a training matter)
            out.extend(_enc_nodes(n.kwargs['body']))
            continue
        if n.kind == 'py':
            raise ValueError("programs with py_func nodes cannot be serialised")
        d = {'k': n.kind, 'o': n.outs, 'a': _enc(list(n.args))}
        if n.kind == 'torch':
            d['f'] = target_name(n.target)
            d['kw'] = _enc(dict(n.kwargs))
            d['m'] = n.meta
        elif n.kind == 'cond':
            t_nodes, t_refs, f_nodes, f_refs = n.kwargs['branches']
            d['br'] = [_enc_nodes(t_nodes), _enc(list(t_refs)), _enc_nodes(f_nodes), _enc(list(f_refs))]
        elif n.kind == 'while':
            c_nodes, c_ref = n.kwargs['cond']
            b_nodes, b_refs = n.kwargs['body']
            d['carried'] = n.kwargs['carried']
            d['cond'] = [_enc_nodes(c_nodes), _enc(c_ref)]
            d['body'] = [_enc_nodes(b_nodes), _enc(list(b_refs))]
        out.append(d)
    return out


def _dec_nodes(items):
    nodes = []
    for d in items:
        k = d['k']
        args = _dec(d['a'])
        if k == 'torch':
            nodes.append(Node('torch', resolve_target(d['f']), args, _dec(d['kw']), d['o'], d.get('m', {})))
        elif k == 'cond':
            t, tr, f, fr = d['br']
            nodes.append(Node('cond', None, args, {'branches': (_dec_nodes(t), _dec(tr), _dec_nodes(f), _dec(fr))},
                              d['o']))
        elif k == 'while':
            nodes.append(Node('while', None, args, {'carried': d['carried'],
                                                    'cond': (_dec_nodes(d['cond'][0]), _dec(d['cond'][1])),
                                                    'body': (_dec_nodes(d['body'][0]), _dec(d['body'][1]))},
                              d['o']))
        else:
            raise ValueError(f"unknown node kind {k}")
    return nodes


# ----------------------------------------------------------------- programs to/from files
def _fetch_vids(prog, fetch_vars):
    return [_vid_of(prog, v) for v in fetch_vars]


def _pd_export(prog, feed_names, fetch_vids):
    """Reference ProgramDesc bytes (static/pdmodel.py) or None when the program uses an operator
    outside the exportable set (or PADDLE_AMD_PDMODEL=0): then this framework's IR is written."""
    if not pa_flag('pdmodel'):
        return None
    from . import pdmodel
    try:
        data, params = pdmodel.export(prog, feed_names, fetch_vids)
    except pdmodel.Unsupported:
        prog._pd_params = None
        return None
    prog._pd_params = params
    return data


def serialize_program(feed_vars, fetch_vars, program=None, **kw):
    prog = program or default_main_program()
    feed_names = [v.name if isinstance(v, Tensor) else v for v in feed_vars]
    pd = _pd_export(prog, feed_names, _fetch_vids(prog, fetch_vars))
    if pd is not None:
        return pd
    feeds = []
    for name in feed_names:
        vid, shape, dt = prog.feeds[name]
        feeds.append({'name': name, 'vid': vid, 'shape': shape, 'dtype': str(dt).replace('torch.', '')})
    doc = {'format': 'paddle_amd.program/1', 'feeds': feeds, 'fetch': _fetch_vids(prog, fetch_vars),
           'nodes': _enc_nodes(prog.nodes),
           'symbolic': 1 if getattr(prog, '_symbolic', False) else 0,
           'symvals': [[k, e.to_json()] for k, e in getattr(prog, '_symvals', {}).items()],
           'consts': {str(cid): (prog._const_owner.get(cid).name if getattr(prog, '_const_owner', {}).get(cid)
                                 is not None else None) for cid in prog.consts}}
    return json.dumps(doc).encode()


def serialize_persistables(feed_vars, fetch_vars, executor=None, program=None, **kw):
    from safetensors.torch import save
    prog = program or default_main_program()
    if getattr(prog, '_pd_params', None) is None and pa_flag('pdmodel'):
        feed_names = [v.name if isinstance(v, Tensor) else v for v in feed_vars]
        _pd_export(prog, feed_names, _fetch_vids(prog, fetch_vars))
    if getattr(prog, '_pd_params', None) is not None:  # reference .pdiparams: LoDTensor streams
        from .proto import save_combine
        return save_combine([(n, t.detach()) for n, t in prog._pd_params])
    return save({f"c{cid}": t.detach().contiguous().cpu() for cid, t in prog.consts.items()})


def save_inference_model(path_prefix, feed_vars, fetch_vars, executor=None, program=None, **kwargs):
    feed_vars = feed_vars if isinstance(feed_vars, (list, tuple)) else [feed_vars]
    fetch_vars = fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars]
    d = os.path.dirname(path_prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    if _pir_mode(kwargs) and save_pir(feed_vars, fetch_vars, path_prefix, program):
        return
    with open(path_prefix + '.pdmodel', 'wb') as f:
        f.write(serialize_program(feed_vars, fetch_vars, program))
    with open(path_prefix + '.pdiparams', 'wb') as f:
        f.write(serialize_persistables(feed_vars, fetch_vars, executor, program))


class LoadedProgram(Program):
    """A Program rebuilt from files; fetch targets are placeholder Variables."""

    def __init__(self):
        super().__init__()
        self._symbolic = False  # set by the loader when the file carries its dim expressions


def deserialize_program(data, device=None):
    from . import pdmodel, pir_json
    with _paused():
        if isinstance(data, (bytes, bytearray)) and pdmodel.is_program_desc(bytes(data[:1])):
            return pdmodel.load(bytes(data))
        if pir_json.is_pir_json(data):  # the reference's PIR .json program (save_pir)
            return pir_json.load(data)
        return _deserialize_program(data, device)


def _pir_mode(kwargs):
    """Write the reference's PIR .json program instead of a ProgramDesc: format='pir' /
    FLAGS_enable_pir_api (the reference 3.x default) / PADDLE_AMD_PIR=1."""
    fmt = kwargs.get('format')
    if fmt is not None:
        return str(fmt).lower() in ('pir', 'json')
    if pa_flag('pir') != '':
        return str(pa_flag('pir')) == '1'
    try:
        from ..framework.flags import get_flags
        return bool(get_flags(['FLAGS_enable_pir_api']).get('FLAGS_enable_pir_api', False))
    except Exception:  # noqa: BLE001
        return False


def save_pir(feed_vars, fetch_vars, path_prefix, program=None):
    """<prefix>.json (PIR program) + <prefix>.pdiparams; returns False when the program uses an
    operator outside the lowered set (the caller then writes the other format)."""
    from . import pdmodel, pir_json
    prog = program or default_main_program()
    feed_names = [v.name if isinstance(v, Tensor) else v for v in feed_vars]
    try:
        data, params = pir_json.export(prog, feed_names, _fetch_vids(prog, fetch_vars))
    except pdmodel.Unsupported:
        return False
    from .proto import save_combine
    with open(path_prefix + '.json', 'wb') as f:
        f.write(data)
    with open(path_prefix + '.pdiparams', 'wb') as f:
        f.write(save_combine([(n, t.detach()) for n, t in params]))
    return True


def _deserialize_program(data, device=None):
    doc = json.loads(data.decode() if isinstance(data, (bytes, bytearray)) else data)
    prog = LoadedProgram()
    prog.nodes = _dec_nodes(doc['nodes'])
    if doc.get('symbolic'):  # dims as expressions; files without it re-specialise by factoring
        prog._symbolic = True
        prog._symvals = {int(k): _sym.expr_from_json(e) for k, e in doc.get('symvals', [])}
    for fd in doc['feeds']:
        prog.feeds[fd['name']] = (fd['vid'], fd['shape'], _DTYPES[fd['dtype']])
        m = torch.empty([max(s, 1) for s in fd['shape']], dtype=_DTYPES[fd['dtype']], device='meta')
        prog._val[id(m)] = fd['vid']
        prog._keep.append(m)
        v = _wrap(m)
        v._name = fd['name']
        prog.named_vars[fd['name']] = v
    prog._fetch = doc['fetch']
    prog._const_names = {int(k): v for k, v in doc['consts'].items()}
    prog._fetch_vars = []
    for vid in doc['fetch']:
        m = torch.empty(0, device='meta')
        prog._val[id(m)] = vid
        prog._keep.append(m)
        prog._fetch_vars.append(_wrap(m))
    return prog


def deserialize_persistables(program, data, executor=None, device=None):
    from safetensors.torch import load
    from ..core.place import current_device
    from ..core.tensor import Parameter
    dev = device or current_device()
    if getattr(program, '_pdmodel', False):
        from . import pdmodel
        pdmodel.load_params(program, data, dev)
        return
    tensors = load(data)
    program._const_owner = {}
    for cid, name in program._const_names.items():
        t = tensors[f"c{cid}"].to(dev)
        if name is not None:
            p = Parameter(t, trainable=t.is_floating_point(), name=name)
            program.consts[cid] = p._t
            program._const_owner[cid] = p
        else:
            program.consts[cid] = t
            program._const_owner[cid] = None


def load_inference_model(path_prefix, executor=None, **kwargs):
    """Returns [program, feed_target_names, fetch_targets]."""
    from ..core.place import to_device
    dev = executor._dev if executor is not None and hasattr(executor, '_dev') else to_device(None)
    model = path_prefix + '.json' if os.path.exists(path_prefix + '.json') and \
        not os.path.exists(path_prefix + '.pdmodel') else path_prefix + '.pdmodel'
    with open(model, 'rb') as f:
        prog = deserialize_program(f.read(), dev)
    with open(path_prefix + '.pdiparams', 'rb') as f:
        deserialize_persistables(prog, f.read(), executor, dev)
    return [prog, list(prog.feeds.keys()), prog._fetch_vars]


# ----------------------------------------------------------------- parameter state
def save(program, model_path, protocol=4, **configs):
    """static.save: parameters of ``program`` to ``<model_path>.pdparams`` (paddle.save format)."""
    from ..framework.io import save as psave
    state = {p.name: p for p in program.all_parameters()}
    psave(state, model_path + '.pdparams', protocol=protocol)


def load(program, model_path, executor=None, var_list=None):
    from ..framework.io import load as pload
    path = model_path if model_path.endswith('.pdparams') else model_path + '.pdparams'
    state = pload(path)
    set_program_state(program, state)


def load_program_state(model_path, var_list=None):
    from ..framework.io import load as pload
    path = model_path if model_path.endswith('.pdparams') else model_path + '.pdparams'
    return pload(path)


def set_program_state(program, state_dict):
    import numpy as np
    for p in program.all_parameters():
        if p.name in state_dict:
            v = state_dict[p.name]
            src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            with torch.no_grad():
                p._t.copy_(src.to(p._t.device, p._t.dtype))


# ----------------------------------------------------------------- paddle.load fallbacks
def load_binary_object(data):
    """paddle.load of a non-pickle file: a serialized Program (returns it) or None."""
    try:
        return deserialize_program(data)
    except Exception:  # noqa: BLE001 - not a program either
        return None


def load_persistables_dir(path, **configs):
    """paddle.load on a directory / path prefix: the parameters saved by save_inference_model or
    jit.save under that prefix, as a {name: Tensor} state dict."""
    prefix = path[:-len('.pdiparams')] if str(path).endswith('.pdiparams') else str(path)
    for cand in (prefix, os.path.join(prefix, 'model'), os.path.join(prefix, '__model__')):
        if os.path.exists(cand + '.pdmodel') and os.path.exists(cand + '.pdiparams'):
            with open(cand + '.pdmodel', 'rb') as f:
                prog = deserialize_program(f.read())
            with open(cand + '.pdiparams', 'rb') as f:
                deserialize_persistables(prog, f.read())
            out = {}
            for cid, name in prog._const_names.items():
                if name is not None:
                    out[name] = prog._const_owner[cid]
            return out
    raise ValueError(f"`paddle.load` can not parse the file: {path} (no such file or saved model prefix)")
