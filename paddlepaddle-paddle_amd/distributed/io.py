"""paddle.distributed.io (reference: python/paddle/distributed/io.py:132 load_persistables,
:357 is_persistable, :392 save_persistables, :464 load_inference_model_distributed).

Persistable variables of a static Program (its parameters) are written in the reference's
LoDTensor stream format (static/proto.py): one file per variable named after it, or all of them
in one ``filename`` in sorted-name order (the save_combine layout of a ``.pdiparams``), so the
directories interoperate with the reference's save_vars / load_vars.
"""
import os

import torch

from ..core.tensor import Tensor, Parameter
from ..static import proto

__all__ = ['save_persistables', 'load_persistables', 'is_persistable', 'load_inference_model_distributed']


def is_persistable(var):
    """True for parameters and variables marked persistable (feed / fetch / reader vars are not)."""
    if isinstance(var, Parameter):
        return True
    return bool(getattr(var, 'persistable', False))


def _persistables(main_program):
    from ..static import default_main_program
    prog = main_program or default_main_program()
    return {p.name: p for p in prog.all_parameters() if is_persistable(p)}


def save_persistables(executor, dirname, main_program=None, filename=None):
    params = _persistables(main_program)
    os.makedirs(dirname, exist_ok=True)
    if filename:
        with open(os.path.join(dirname, filename), 'wb') as f:
            f.write(proto.save_combine([(n, p._t) for n, p in params.items()]))
        return
    for n, p in params.items():
        with open(os.path.join(dirname, n), 'wb') as f:
            f.write(proto.tensor_to_stream(p._t))


def load_persistables(executor, dirname, main_program=None, filename=None):
    params = _persistables(main_program)
    if filename:
        with open(os.path.join(dirname, filename), 'rb') as f:
            vals = proto.load_combine(f.read(), list(params))
    else:
        vals = {}
        for n in params:
            with open(os.path.join(dirname, n), 'rb') as f:
                vals[n], _ = proto.tensor_from_stream(f)
    with torch.no_grad():
        for n, p in params.items():
            v = vals[n]
            if tuple(v.shape) != tuple(p._t.shape):
                raise ValueError(f"load_persistables: {n} has shape {tuple(v.shape)} in {dirname}, "
                                 f"expected {tuple(p._t.shape)}")
            p._t.copy_(v.to(p._t.device, p._t.dtype))


def load_inference_model_distributed(dirname, executor, model_filename=None, params_filename=None,
                                     pserver_endpoints=None):
    """[program, feed_target_names, fetch_targets] of an inference model saved under ``dirname``
    (``model_filename`` / ``params_filename`` name the two files; a path prefix also works)."""
    from ..static.io import load_inference_model
    if model_filename is not None:
        prefix = os.path.join(dirname, os.path.splitext(model_filename)[0])
    elif os.path.isdir(dirname):
        prefix = os.path.join(dirname, 'model')
    else:
        prefix = dirname
    return load_inference_model(prefix, executor)
