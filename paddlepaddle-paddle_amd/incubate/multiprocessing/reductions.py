"""Shared-memory pickling of paddle Tensors across worker processes
(reference: python/paddle/incubate/multiprocessing/reductions.py — file_system strategy,
``_reduce_tensor`` / ``_rebuild_*`` registered on ``ForkingPickler``).

A paddle Tensor here is a thin handle over a storage-layer tensor, so the handle is pickled as
(storage tensor, paddle attributes) and the storage tensor travels through the storage layer's own
multiprocessing reductions: a CPU tensor's storage is moved into shared memory (file-descriptor or
file-system strategy) and the receiving process maps the same pages — a write on either side is seen
by the other; a GPU tensor crosses as a device IPC handle (dmabuf on this platform), the producer
keeping the allocation alive.  Parameters keep their trainable / name attributes.
"""
from multiprocessing.reduction import ForkingPickler

import torch
import torch.multiprocessing as _tmp  # noqa: F401  (registers the storage-layer reductions)


def _supported_check():
    import sys
    if not sys.platform.startswith('linux'):
        return False
    return True


def _rebuild_tensor(cls_name, t, stop_gradient, name, attrs):
    from ...core.tensor import Tensor, Parameter
    if cls_name == 'Parameter':
        p = Parameter(t, trainable=attrs.get('_trainable', True), name=name)
        for k, v in attrs.items():
            p.__dict__[k] = v
        return p
    out = Tensor(t, name=name)
    if not stop_gradient and t.is_floating_point():
        out._t.requires_grad_(True)
    return out


def _reduce_tensor(tensor):
    t = tensor._t
    if t.is_meta:
        raise RuntimeError("a static-graph Variable (meta tensor) cannot be shared across processes")
    base = t.detach()
    if not base.is_cuda:
        base = base.share_memory_() if not base.is_shared() else base
    attrs = {}
    if type(tensor).__name__ == 'Parameter':
        attrs = {k: v for k, v in tensor.__dict__.items() if k in ('_trainable', 'need_clip', 'is_distributed',
                                                                   'optimize_attr', 'do_model_average')}
    return _rebuild_tensor, (type(tensor).__name__, base, not t.requires_grad, tensor._name, attrs)


_done = [False]


def init_reductions():
    if not _supported_check() or _done[0]:
        return
    from ...core.tensor import Tensor, Parameter
    ForkingPickler.register(Tensor, _reduce_tensor)
    ForkingPickler.register(Parameter, _reduce_tensor)
    _done[0] = True


_ = torch
