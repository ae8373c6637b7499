"""paddle.nn.Layer (reference: python/paddle/nn/layer/layers.py:332).

Parameters are leaf storage tensors on the current HIP device wrapped as ``Parameter``;
sublayers / parameters / buffers live in ordered dicts exactly like the reference so that
``state_dict`` keys (structured names such as ``encoder.layers.0.linear1.weight``) match
checkpoints written by the reference.
"""
import collections
import re

import numpy as np
import torch

from ...core import dtype as _dt
from ...core.tensor import Tensor, Parameter, _wrap, _unwrap
from ...core.place import current_device, to_device
from ...framework.param_attr import ParamAttr
from ...utils import unique_name
from .. import initializer as I
from ...core.tensor import register_param as _register_param


def _camel_to_snake(name):
    s1 = re.sub('(.)([A-Z][a-z]+)', r'\1_\2', name)
    return re.sub('([a-z0-9])([A-Z])', r'\1_\2', s1).lower()


def _create_parameter(shape, dtype=None, attr=None, is_bias=False, default_initializer=None, name=None,
                      prefix='param'):
    attr = ParamAttr._to_attr(attr)
    if attr is False:
        return None
    dtype = _dt.to_torch_dtype(dtype) if dtype is not None else _dt.default_float()
    t = torch.empty([int(s) for s in shape], dtype=dtype, device=current_device())
    init = attr.initializer or I._global_init(is_bias) or default_initializer
    if init is None:
        init = I.Constant(0.0) if is_bias else I.XavierUniform()
    with torch.no_grad():
        init._init(t)
    p = Parameter(t, trainable=attr.trainable, name=attr.name or name or unique_name.generate(prefix + ('.b' if is_bias else '.w')),
                  optimize_attr={'learning_rate': attr.learning_rate}, regularizer=attr.regularizer,
                  need_clip=attr.need_clip, do_model_average=attr.do_model_average)
    return p


class HookRemoveHelper:
    next_hook_id = 0

    def __init__(self, hooks, extra_hook_dict=None):
        self._hooks_ref = hooks
        self._hook_id = HookRemoveHelper.next_hook_id
        HookRemoveHelper.next_hook_id += 1

    def remove(self):
        self._hooks_ref.pop(self._hook_id, None)


class Layer:
    """Base class of all layers (dygraph)."""

    def __init__(self, name_scope=None, dtype='float32'):
        d = self.__dict__
        d['training'] = True
        d['_parameters'] = collections.OrderedDict()
        d['_sub_layers'] = collections.OrderedDict()
        d['_buffers'] = collections.OrderedDict()
        d['_non_persistable_buffer_names_set'] = set()
        d['_forward_pre_hooks'] = collections.OrderedDict()
        d['_forward_post_hooks'] = collections.OrderedDict()
        d['_dtype'] = dtype
        d['_full_name'] = unique_name.generate(name_scope or _camel_to_snake(self.__class__.__name__))
        d['_built'] = False
        d['_casted_by_pure_fp16'] = False
        d['_state_dict_hooks'] = collections.OrderedDict()
        d['_load_state_dict_pre_hooks'] = collections.OrderedDict()

    # ------------------------------------------------------------------ attribute routing
    def __setattr__(self, name, value):
        d = self.__dict__
        params = d.get('_parameters')
        if isinstance(value, Parameter):
            if params is None:
                raise ValueError("super().__init__() must be called before assigning parameters")
            d.get('_sub_layers', {}).pop(name, None)
            d.get('_buffers', {}).pop(name, None)
            d.pop(name, None)
            params[name] = value
            return
        if isinstance(value, Layer):
            if params is None:
                raise ValueError("super().__init__() must be called before assigning sublayers")
            params.pop(name, None)
            d['_buffers'].pop(name, None)
            d.pop(name, None)
            d['_sub_layers'][name] = value
            return
        if params is not None and name in params:
            if value is None:
                params[name] = None
                return
            if isinstance(value, Tensor):
                params[name] = value if isinstance(value, Parameter) else Parameter(value, trainable=not value.stop_gradient)
                return
            raise TypeError(f"assigning {type(value)} to parameter '{name}'")
        bufs = d.get('_buffers')
        if bufs is not None and name in bufs:
            if value is None or isinstance(value, Tensor):
                bufs[name] = value
                return
        subs = d.get('_sub_layers')
        if subs is not None and name in subs and value is None:
            subs[name] = None
            return
        object.__setattr__(self, name, value)

    def __getattr__(self, name):
        d = self.__dict__
        for k in ('_parameters', '_sub_layers', '_buffers'):
            store = d.get(k)
            if store is not None and name in store:
                return store[name]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")

    def __delattr__(self, name):
        for k in ('_parameters', '_sub_layers', '_buffers'):
            if name in self.__dict__.get(k, {}):
                del self.__dict__[k][name]
                return
        object.__delattr__(self, name)

    def __dir__(self):
        return list(super().__dir__()) + list(self._parameters) + list(self._sub_layers) + list(self._buffers)

    # ------------------------------------------------------------------ construction helpers
    def full_name(self):
        return self._full_name

    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False, default_initializer=None):
        dtype = dtype if dtype is not None else self._dtype
        return _create_parameter(shape, dtype, attr, is_bias, default_initializer, prefix=self._full_name)

    def create_variable(self, name=None, persistable=None, dtype=None):
        t = _wrap(torch.empty(0, dtype=_dt.to_torch_dtype(dtype or self._dtype), device=current_device()))
        t.persistable = bool(persistable)
        return t

    create_tensor = create_variable

    def add_parameter(self, name, parameter):
        if parameter is not None and not isinstance(parameter, Parameter):
            raise TypeError("add_parameter expects a Parameter")
        self._parameters[name] = parameter
        return parameter

    def add_sublayer(self, name, sublayer):
        self._sub_layers[str(name)] = sublayer
        return sublayer

    def register_buffer(self, name, tensor, persistable=True):
        if tensor is not None and not isinstance(tensor, Tensor):
            tensor = _wrap(torch.as_tensor(np.asarray(tensor)))
        self._buffers[name] = tensor
        if persistable:
            self._non_persistable_buffer_names_set.discard(name)
        else:
            self._non_persistable_buffer_names_set.add(name)
        if tensor is not None:
            tensor.persistable = persistable

    # ------------------------------------------------------------------ iteration
    def named_parameters(self, prefix='', include_sublayers=True, remove_duplicate=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, layer in layers:
            for n, p in layer._parameters.items():
                if p is None or (remove_duplicate and id(p) in seen):
                    continue
                seen.add(id(p))
                yield (lp + '.' + n if lp else n), p

    def parameters(self, include_sublayers=True):
        return [p for _, p in self.named_parameters(include_sublayers=include_sublayers)]

    def named_sublayers(self, prefix='', include_self=False, layers_set=None):
        if layers_set is None:
            layers_set = set()
        if include_self and id(self) not in layers_set:
            layers_set.add(id(self))
            yield prefix, self
        for name, layer in self._sub_layers.items():
            if layer is None:
                continue
            p = prefix + ('.' if prefix else '') + name
            if id(layer) in layers_set:
                continue
            layers_set.add(id(layer))
            yield p, layer
            yield from layer.named_sublayers(prefix=p, include_self=False, layers_set=layers_set)

    def sublayers(self, include_self=False):
        return [l for _, l in self.named_sublayers(include_self=include_self)]

    def named_children(self):
        for n, l in self._sub_layers.items():
            if l is not None:
                yield n, l

    def children(self):
        return [l for _, l in self.named_children()]

    def named_buffers(self, prefix='', include_sublayers=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, layer in layers:
            for n, b in layer._buffers.items():
                if b is None or id(b) in seen:
                    continue
                seen.add(id(b))
                yield (lp + '.' + n if lp else n), b

    def buffers(self, include_sublayers=True):
        return [b for _, b in self.named_buffers(include_sublayers=include_sublayers)]

    # ------------------------------------------------------------------ modes
    def train(self):
        for l in self.sublayers(include_self=True):
            l.__dict__['training'] = True
        return self

    def eval(self):
        for l in self.sublayers(include_self=True):
            l.__dict__['training'] = False
        return self

    # ------------------------------------------------------------------ call
    def forward(self, *inputs, **kwargs):
        raise NotImplementedError

    def __call__(self, *inputs, **kwargs):
        pre = self.__dict__['_forward_pre_hooks']
        if pre:
            for h in list(pre.values()):
                r = h(self, inputs)
                if r is not None:
                    inputs = r if isinstance(r, tuple) else (r,)
        out = self.forward(*inputs, **kwargs)
        post = self.__dict__['_forward_post_hooks']
        if post:
            for h in list(post.values()):
                r = h(self, inputs, out)
                if r is not None:
                    out = r
        return out

    def register_forward_pre_hook(self, hook):
        h = HookRemoveHelper(self._forward_pre_hooks)
        self._forward_pre_hooks[h._hook_id] = hook
        return h

    def register_forward_post_hook(self, hook):
        h = HookRemoveHelper(self._forward_post_hooks)
        self._forward_post_hooks[h._hook_id] = hook
        return h

    def apply(self, fn):
        for l in self.children():
            l.apply(fn)
        fn(self)
        return self

    def clear_gradients(self, set_to_zero=True):
        for p in self.parameters():
            if p.trainable:
                p.clear_grad(set_to_zero=set_to_zero)

    clear_grad = clear_gradients

    # ------------------------------------------------------------------ state
    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix='', use_hook=True,
                   keep_vars=True):
        dest = collections.OrderedDict() if destination is None else destination
        for n, p in self._parameters.items():
            if p is not None:
                dest[structured_name_prefix + n] = p
        for n, b in self._buffers.items():
            if b is not None and n not in self._non_persistable_buffer_names_set:
                dest[structured_name_prefix + n] = b
        if include_sublayers:
            for ln, l in self._sub_layers.items():
                if l is not None:
                    l.state_dict(dest, True, structured_name_prefix + ln + '.', use_hook)
        if use_hook:
            for h in self._state_dict_hooks.values():
                r = h(dest)
                if r is not None:
                    dest = r
        return dest

    to_static_state_dict = state_dict

    def register_state_dict_hook(self, hook):
        h = HookRemoveHelper(self._state_dict_hooks)
        self._state_dict_hooks[h._hook_id] = hook
        return h

    def set_state_dict(self, state_dict, use_structured_name=True):
        own = self.state_dict(use_hook=False)
        if not use_structured_name:
            by_name = {v.name: k for k, v in own.items()}
        missing, unexpected = [], []
        matched = set()
        for k, v in state_dict.items():
            key = k if use_structured_name else by_name.get(k)
            if key is None or key not in own:
                unexpected.append(k)
                continue
            tgt = own[key]
            if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str):  # (name, ndarray) pickle form
                v = v[1]
            src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            if isinstance(v, np.ndarray) and v.dtype == np.uint16 and tgt.dtype == torch.bfloat16:
                src = torch.from_numpy(v.view(np.int16)).view(torch.bfloat16)
            if list(src.shape) != tgt.shape:
                raise ValueError(f"shape mismatch for {key}: {list(src.shape)} vs {tgt.shape}")
            with torch.no_grad():
                tgt._t.copy_(src.to(tgt._t.dtype))
            matched.add(key)
        missing = [k for k in own if k not in matched]
        return missing, unexpected

    set_dict = set_state_dict
    load_dict = set_state_dict

    # ------------------------------------------------------------------ dtype / device
    def _apply_tensors(self, fn, floating_only=True):
        for l in self.sublayers(include_self=True):
            for n, p in l._parameters.items():
                if p is None or (floating_only and not p._t.is_floating_point()):
                    continue
                with torch.no_grad():
                    new = fn(p._t.detach())
                req = p._t.requires_grad
                p._t = new.detach().requires_grad_(req)
                _register_param(p)
            for n, b in l._buffers.items():
                if b is None or (floating_only and not b._t.is_floating_point()):
                    continue
                b._t = fn(b._t)
        return self

    def to(self, device=None, dtype=None, blocking=None, floating_only=True):
        dev = to_device(device) if device is not None else None
        dt = _dt.to_torch_dtype(dtype)

        def fn(t):
            if dev is not None:
                t = t.to(dev)
            if dt is not None and t.is_floating_point():
                t = t.to(dt)
            return t
        self._apply_tensors(fn, floating_only=False)
        if dt is not None:
            for l in self.sublayers(include_self=True):
                l.__dict__['_dtype'] = _dt.dtype_name(dt)
        return self

    def astype(self, dtype=None):
        return self.to(dtype=dtype)

    def float(self, excluded_layers=None):
        return self.to(dtype='float32')

    def float16(self, excluded_layers=None):
        return self.to(dtype='float16')

    def bfloat16(self, excluded_layers=None):
        return self.to(dtype='bfloat16')

    half = float16

    def cuda(self, device=None):
        return self.to(device=device if device is not None else 'gpu')

    def cpu(self):
        return self.to(device='cpu')

    # ------------------------------------------------------------------ repr
    def extra_repr(self):
        return ''

    def __repr__(self):
        lines = []
        for n, l in self._sub_layers.items():
            mod = repr(l).replace('\n', '\n  ')
            lines.append(f"({n}): {mod}")
        main = self.__class__.__name__ + '(' + self.extra_repr()
        if lines:
            main += '\n  ' + '\n  '.join(lines) + '\n'
        return main + ')'

    def __getstate__(self):
        return self.__dict__

    def __setstate__(self, state):
        self.__dict__.update(state)
