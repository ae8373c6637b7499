"""fp32 main-gradient training of a low-precision (bf16 / fp16) model (reference:
python/paddle/distributed/fleet/utils/mix_precision_utils.py — MixPrecisionLayer:35,
MixPrecisionOptimizer:97, MixPrecisionScaler:244).

``MixPrecisionLayer`` gives every parameter an fp32 ``main_grad``: a post-accumulate hook adds each
low-precision gradient into it and releases the low-precision one, so gradient accumulation over
micro-batches happens in fp32.  ``MixPrecisionOptimizer`` steps the wrapped optimizer on the
``main_grad`` s (its fp32 master weights, when multi_precision, receive fp32 gradients) and
``clear_grad`` zeroes / drops them.  ``MixPrecisionScaler`` unscales ``main_grad`` in place."""
import torch

from ....core.tensor import Tensor, _wrap
from ....nn.layer.layers import Layer


class MixPrecisionLayer(Layer):
    def __init__(self, layers, dtype="float16"):
        super().__init__()
        assert dtype in ("float16", "bfloat16"), dtype
        self._layers = layers
        self._dtype = dtype
        self._hooks = []
        for p in layers.parameters():
            if 'main_grad' not in p.__dict__:
                p.__dict__['main_grad'] = None
                if p._t.requires_grad:
                    self._hooks.append(p._t.register_post_accumulate_grad_hook(self._update_main_grad_hook(p)))

    @staticmethod
    def _update_main_grad_hook(param):
        @torch.no_grad()
        def hook(t):
            g = t.grad
            if g is None:
                return
            mg = param.__dict__.get('main_grad')
            if mg is None:
                param.__dict__['main_grad'] = _wrap(g.float().clone())
            else:
                mg._t.add_(g.float())
            t.grad = None
        return hook

    def forward(self, *inputs, **kwargs):
        return self._layers(*inputs, **kwargs)

    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix=""):
        return self._layers.state_dict()

    def set_state_dict(self, state_dict, use_structured_name=True):
        return self._layers.set_state_dict(state_dict, use_structured_name)


class MixPrecisionOptimizer:
    def __init__(self, optimizer):
        self._inner_opt = optimizer
        self._parameter_list = list(optimizer._parameter_list)

    @torch.no_grad()
    def step(self):
        opt = self._inner_opt
        lr = opt.get_lr()
        for group in opt._param_groups:
            pg = []
            for p in group['params']:
                mg = p.__dict__.get('main_grad')
                if not p.trainable or mg is None:
                    continue
                pg.append((p, mg))
            if not pg:
                continue
            clip = group.get('grad_clip', opt._grad_clip)
            if clip is not None:
                pg = clip(pg)
            opt._update_group(group, pg, lr * group.get('learning_rate', 1.0))
        opt._global_step += 1

    def clear_grad(self, set_to_zero=True):
        for p in self._parameter_list:
            mg = p.__dict__.get('main_grad')
            if mg is None:
                continue
            if set_to_zero:
                mg._t.zero_()
            else:
                p.__dict__['main_grad'] = None
            p._t.grad = None

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def __getattr__(self, item):
        return getattr(self.__dict__['_inner_opt'], item)


def unscale_method(self, optimizer):
    """GradScaler.unscale_ for main-grad training: divide every fp32 main_grad by the scale and
    record found_inf (reference mix_precision_utils.unscale_method:201)."""
    if not self._enable:
        return
    inv = 1.0 / float(self._scale)
    found = False
    params = optimizer._parameter_list if hasattr(optimizer, '_parameter_list') else []
    for p in params:
        mg = p.__dict__.get('main_grad')
        if mg is None:
            continue
        mg._t.mul_(inv)
        if not bool(torch.isfinite(mg._t).all()):
            found = True
    self._found_inf = found


class MixPrecisionScaler:
    def __init__(self, scaler):
        self._inner = scaler
        import types
        scaler._unscale = types.MethodType(unscale_method, scaler)

    def __getattr__(self, item):
        return getattr(self.__dict__['_inner'], item)
