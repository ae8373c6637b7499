"""paddle.onnx.export (reference: python/paddle/onnx/export.py:22 — delegates to paddle2onnx).

paddle2onnx and the ``onnx`` package are not available here, so the graph is emitted by
PyTorch's TorchScript ONNX exporter (C++ graph lowering + protobuf serialisation inside libtorch)
over a trace of the Layer's forward on the non-HIP path: the custom HIP kernels are launched
through ctypes and are not traceable, so export runs with them disabled and the graph is built
from the equivalent decomposed torch ops (LayerNorm/Softmax/Gemm/... ONNX nodes).  ``None`` dims of
the InputSpecs become dynamic axes.  ``inspect`` decodes the written ModelProto (wire format, no
onnx package needed) for checks.
"""
import contextlib
import os

import torch

_OPSET_MIN = 13  # the reference's default 9 predates LayerNormalization-era decompositions


class _Adapter(torch.nn.Module):
    def __init__(self, layer):
        super().__init__()
        self._layer = layer

    def forward(self, *xs):
        from .core.tensor import _wrap, _unwrap
        out = self._layer(*[_wrap(x) for x in xs])
        if isinstance(out, (list, tuple)):
            return tuple(_unwrap(o) for o in out)
        return _unwrap(out)


def _example(spec, i):
    """(example tensor, dynamic dim indices, input name) of one InputSpec / Tensor."""
    from .core.tensor import Tensor, _unwrap
    from .core import dtype as _dt
    if isinstance(spec, Tensor):
        return _unwrap(spec).detach(), [], getattr(spec, 'name', None) or f"x{i}"
    if isinstance(spec, torch.Tensor):
        return spec.detach(), [], f"x{i}"
    shape = [1 if (s is None or s < 0) else int(s) for s in spec.shape]
    dt = _dt.to_torch_dtype(spec.dtype) if spec.dtype is not None else torch.float32
    x = torch.randn(shape).to(dt) if dt.is_floating_point else torch.zeros(shape, dtype=dt)
    dyn = [j for j, s in enumerate(spec.shape) if s is None or s < 0]
    return x, dyn, spec.name or f"x{i}"


@contextlib.contextmanager
def _no_onnx_package():
    """The TorchScript exporter imports ``onnx`` only to splice onnx-script custom functions
    into the ModelProto; we export none, so the serialized bytes are final."""
    try:
        import onnx  # noqa: F401
        yield
        return
    except ImportError:
        pass
    from torch.onnx._internal.torchscript_exporter import onnx_proto_utils as opu
    orig = opu._add_onnxscript_fn
    opu._add_onnxscript_fn = lambda model_bytes, custom_opsets: model_bytes
    try:
        yield
    finally:
        opu._add_onnxscript_fn = orig


def export(layer, path, input_spec=None, opset_version=9, **configs):
    """Writes ``path + '.onnx'`` (reference contract) and returns the file name."""
    from . import ops
    if input_spec is None:
        raise ValueError("paddle.onnx.export needs input_spec (InputSpec or example Tensors)")
    examples = [_example(s, i) for i, s in enumerate(input_spec)]
    args = tuple(e[0] for e in examples)
    names = [e[2] for e in examples]
    dynamic_axes = {name: {j: f"{name}_d{j}" for j in dyn} for (_, dyn, name) in examples if dyn}
    out_file = path if path.endswith('.onnx') else path + '.onnx'
    os.makedirs(os.path.dirname(os.path.abspath(out_file)), exist_ok=True)
    was_training = getattr(layer, 'training', False)
    layer.eval()
    # trace on the CPU copy-free path: move nothing, but make sure no HIP kernel is traced
    was_enabled = ops.enabled()
    ops.set_enabled(False)
    params = list(layer.parameters())
    flags = [p._t.requires_grad for p in params]
    try:
        # parameters enter the trace as constants -> ONNX initializers (constant-folded)
        for p in params:
            p._t.requires_grad_(False)
        dev = params[0]._t.device if params else torch.device('cpu')
        args = tuple(a.to(dev) for a in args)
        with _no_onnx_package(), torch.no_grad():
            torch.onnx.export(_Adapter(layer), args, out_file, dynamo=False,
                              opset_version=max(int(opset_version), _OPSET_MIN), input_names=names,
                              dynamic_axes=dynamic_axes or None, do_constant_folding=True)
    finally:
        for p, f in zip(params, flags):
            p._t.requires_grad_(f)
        ops.set_enabled(was_enabled)
        if was_training:
            layer.train()
    return out_file


# ---------------------------------------------------------------- ModelProto inspection
def _varint(b, i):
    v, s = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def _fields(b):
    i, out = 0, []
    while i < len(b):
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.append((f, v))
    return out


def inspect(file_or_bytes):
    """{'opset': int, 'ops': [op_type...], 'inputs': [...], 'outputs': [...], 'initializers': n}"""
    b = open(file_or_bytes, 'rb').read() if isinstance(file_or_bytes, str) else bytes(file_or_bytes)
    model = _fields(b)
    graph = next(v for f, v in model if f == 7)
    opset = [dict(_fields(v)).get(2) for f, v in model if f == 8]
    ops, inputs, outputs, inits = [], [], [], 0
    for f, v in _fields(graph):
        if f == 1:
            ops.append(bytes(dict(_fields(v))[4]).decode())
        elif f == 5:
            inits += 1
        elif f == 11:
            inputs.append(bytes(dict(_fields(v))[1]).decode())
        elif f == 12:
            outputs.append(bytes(dict(_fields(v))[1]).decode())
    return {'opset': opset[0] if opset else None, 'ops': ops, 'inputs': inputs, 'outputs': outputs,
            'initializers': inits}
