"""Model summary (reference: python/paddle/hapi/model_summary.py:29 summary): per-layer
output shapes and parameter counts from forward hooks on one synthetic batch."""
import numpy as np
import torch

from ..core.tensor import Tensor


def _make_inputs(input_size, dtypes, dev):
    from ..core.tensor import _wrap
    if isinstance(input_size, tuple) and all(isinstance(i, (int, type(None))) for i in input_size):
        input_size = [input_size]
    dtypes = dtypes if isinstance(dtypes, (list, tuple)) else [dtypes] * len(input_size)
    xs = []
    for shp, dt in zip(input_size, dtypes):
        if hasattr(shp, 'shape'):
            shp = shp.shape
        shp = [1 if (s is None or s < 0) else s for s in shp]
        from ..core.dtype import to_torch_dtype
        tdt = to_torch_dtype(dt or 'float32')
        t = torch.randint(0, 2, shp, device=dev) if not tdt.is_floating_point else torch.rand(shp, device=dev)
        xs.append(_wrap(t.to(tdt)))
    return xs


def summary(net, input_size=None, dtypes=None, input=None):  # noqa: A002
    from ..core.place import current_device
    rows = []
    hooks = []

    def register(layer):
        def hook(lyr, inp, out):
            o = out[0] if isinstance(out, (list, tuple)) else out
            shape = list(o.shape) if isinstance(o, Tensor) else []
            n = sum(int(np.prod(p.shape)) for p in lyr._parameters.values() if p is not None)
            tr = sum(int(np.prod(p.shape)) for p in lyr._parameters.values() if p is not None and not p.stop_gradient)
            rows.append((f"{type(lyr).__name__}-{len(rows) + 1}", shape, n, tr))
        if not layer._sub_layers or layer._parameters:
            hooks.append(layer.register_forward_post_hook(hook))

    for lyr in net.sublayers(include_self=False) or [net]:
        register(lyr)
    was_training = net.training
    net.eval()
    try:
        with torch.no_grad():
            if input is not None:
                net(*(input if isinstance(input, (list, tuple)) else [input]))
            else:
                net(*_make_inputs(input_size, dtypes, current_device()))
    finally:
        for h in hooks:
            h.remove()
        if was_training:
            net.train()
    total = sum(int(np.prod(p.shape)) for p in net.parameters())
    trainable = sum(int(np.prod(p.shape)) for p in net.parameters() if not p.stop_gradient)
    w = max([len(r[0]) for r in rows] + [12]) + 2
    lines = ['-' * (w + 45), f"{'Layer (type)':<{w}}{'Output Shape':<28}{'Param #':>15}", '=' * (w + 45)]
    for name, shape, n, _ in rows:
        lines.append(f"{name:<{w}}{str(shape):<28}{n:>15,}")
    lines += ['=' * (w + 45), f"Total params: {total:,}", f"Trainable params: {trainable:,}",
              f"Non-trainable params: {total - trainable:,}", '-' * (w + 45)]
    print('\n'.join(lines))
    return {'total_params': total, 'trainable_params': trainable}
