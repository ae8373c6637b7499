"""paddle._C_ops — the generated operator entry points of the reference (python/paddle/_C_ops.py
re-exports paddle/fluid/pybind eager_op_function.cc, one function per op of
paddle/phi/ops/yaml/ops.yaml, positional arguments in the yaml's ``args`` order).

Here each name maps onto this framework's implementation of the same operator (the paddle API
function that runs the hand-written HIP kernel where there is one), with the yaml argument order.
Names without an explicit entry resolve to the paddle / paddle.nn.functional function of the same
name when one exists (the elementwise / unary ops share their signature); anything else raises
AttributeError.
"""
import importlib


def _P():
    return importlib.import_module('paddle')


def _F():
    return importlib.import_module('paddle.nn.functional')


def _IF():
    return importlib.import_module('paddle.incubate.nn.functional')


def _dt(d):
    from .core.dtype import to_torch_dtype
    return d if d is None else to_torch_dtype(d)


def matmul(x, y, transpose_x=False, transpose_y=False):
    return _P().matmul(x, y, transpose_x, transpose_y)


def add(x, y):
    return _P().add(x, y)


def subtract(x, y):
    return _P().subtract(x, y)


def multiply(x, y):
    return _P().multiply(x, y)


def divide(x, y):
    return _P().divide(x, y)


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True):
    return _P().scale(x, scale, bias, bias_after_scale)


def full(shape, value, dtype=None, place=None):
    return _P().full(shape, value, dtype)


def full_like(x, value, dtype=None, place=None):
    return _P().full_like(x, value, dtype)


def cast(x, dtype):
    return _P().cast(x, dtype)


def reshape(x, shape):
    return _P().reshape(x, shape)


def transpose(x, perm):
    return _P().transpose(x, perm)


def concat(x, axis=0):
    return _P().concat(x, axis)


def split(x, sections, axis=0):
    return _P().split(x, sections, axis)


def split_with_num(x, num, axis=0):
    return _P().split(x, num, axis)


def sum(x, axis=None, dtype=None, keepdim=False):  # noqa: A001
    return _P().sum(x, axis if axis not in ([], ()) else None, dtype, keepdim)


def mean(x, axis=None, keepdim=False):
    return _P().mean(x, axis if axis not in ([], ()) else None, keepdim)


def max(x, axis=None, keepdim=False):  # noqa: A001
    return _P().max(x, axis if axis not in ([], ()) else None, keepdim)


def softmax(x, axis=-1):
    return _F().softmax(x, axis)


def log_softmax(x, axis=-1):
    return _F().log_softmax(x, axis)


def gelu(x, approximate=False):
    return _F().gelu(x, approximate)


def silu(x):
    return _F().silu(x)


def swiglu(x, y=None):
    return _F().swiglu(x, y)


def layer_norm(x, scale=None, bias=None, epsilon=1e-5, begin_norm_axis=1):
    """(out, mean, variance) like the reference kernel."""
    import torch
    from .core.tensor import _wrap, _unwrap
    t = _unwrap(x)
    shape = list(t.shape[begin_norm_axis:])
    out = _F().layer_norm(x, shape, scale, bias, epsilon)
    red = tuple(range(begin_norm_axis, t.dim()))
    tf = t.float()
    mean_ = tf.mean(red)
    var = tf.var(red, unbiased=False)
    return out, _wrap(mean_.reshape(-1)), _wrap(var.reshape(-1).to(torch.float32))


def rms_norm(x, bias=None, residual=None, norm_weight=None, norm_bias=None, epsilon=1e-6, begin_norm_axis=-1,
             quant_scale=-1.0, quant_round_type=0, quant_max_bound=0.0, quant_min_bound=0.0):
    r = _IF().fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias, residual)
    return r if isinstance(r, tuple) else (r, None)


def embedding(x, weight, padding_idx=-1, sparse=False):
    return _F().embedding(x, weight, None if padding_idx == -1 else padding_idx, sparse)


def dropout(x, seed_tensor=None, p=0.5, is_test=False, mode='upscale_in_train', seed=0, fix_seed=False):
    return _F().dropout(x, float(p), training=not is_test, mode=mode), None


def flash_attn(q, k, v, fixed_seed_offset=None, attn_mask=None, dropout=0.0, causal=False, return_softmax=False,
               is_test=False, rng_name=''):
    """(out, softmax, softmax_lse, seed_offset) like the reference kernel (softmax / lse: None)."""
    F = _F()
    if attn_mask is not None:
        out = F.scaled_dot_product_attention(q, k, v, attn_mask, dropout, causal, training=not is_test)
    else:
        out = F.flash_attention(q, k, v, dropout, causal, training=not is_test)[0]
    return out, None, None, None


def fused_rotary_position_embedding(q, k=None, v=None, sin=None, cos=None, position_ids=None,
                                    use_neox_rotary_style=True, time_major=False, rotary_emb_base=10000.0):
    return _IF().fused_rotary_position_embedding(q, k, v, sin, cos, position_ids, use_neox_rotary_style, time_major,
                                                 rotary_emb_base)


def conv2d(input, filter, strides=(1, 1), paddings=(0, 0), padding_algorithm='EXPLICIT',  # noqa: A002
           dilations=(1, 1), groups=1, data_format='NCHW'):
    pad = padding_algorithm.lower() if padding_algorithm in ('SAME', 'VALID') else list(paddings)
    return _F().conv2d(input, filter, None, list(strides), pad, list(dilations), groups, data_format)


def pool2d(x, kernel_size, strides, paddings, ceil_mode, exclusive, data_format, pooling_type, global_pooling,
           adaptive, padding_algorithm):
    F = _F()
    if global_pooling or adaptive:
        osz = [1, 1] if global_pooling else kernel_size
        fn = F.adaptive_max_pool2d if pooling_type == 'max' else F.adaptive_avg_pool2d
        return fn(x, osz, data_format=data_format) if pooling_type != 'max' else fn(x, osz)
    if pooling_type == 'max':
        return F.max_pool2d(x, kernel_size, strides, paddings, ceil_mode=ceil_mode, data_format=data_format)
    return F.avg_pool2d(x, kernel_size, strides, paddings, ceil_mode=ceil_mode, exclusive=exclusive,
                        data_format=data_format)


def batch_norm(x, mean, variance, scale, bias, is_test, momentum, epsilon, data_format='NCHW',
               use_global_stats=False, trainable_statistics=False):
    out = _F().batch_norm(x, mean, variance, scale, bias, not is_test, momentum, epsilon, data_format,
                          use_global_stats if use_global_stats else None)
    return out, mean, variance, None, None, None


def cross_entropy_with_softmax(input, label, soft_label=False, use_softmax=True, numeric_stable_mode=True,  # noqa: A002
                               ignore_index=-100, axis=-1):
    F = _F()
    loss = F.cross_entropy(input, label, soft_label=soft_label, ignore_index=ignore_index, reduction='none',
                           axis=axis, use_softmax=use_softmax)
    return F.softmax(input, axis), loss


def adamw_(param, grad, learning_rate, moment1, moment2, moment2_max=None, beta1_pow=None, beta2_pow=None,
           master_param=None, skip_update=None, beta1=0.9, beta2=0.999, epsilon=1e-8, lr_ratio=1.0, coeff=0.01,
           with_decay=True, lazy_mode=False, min_row_size_to_use_multithread=1000, multi_precision=False,
           use_global_beta_pow=False, amsgrad=False):
    """In-place AdamW update of one parameter (the reference's adamw_ kernel contract): param,
    moments, beta powers (and the fp32 master) are updated in place; returns them."""
    import torch
    from .core.tensor import _unwrap
    p, g = _unwrap(param), _unwrap(grad).float()
    m1, m2 = _unwrap(moment1), _unwrap(moment2)
    lr = float(_unwrap(learning_rate).reshape(-1)[0]) if hasattr(learning_rate, 'shape') else float(learning_rate)
    b1p = _unwrap(beta1_pow)
    b2p = _unwrap(beta2_pow)
    master = _unwrap(master_param) if master_param is not None else None
    w = master if master is not None else p
    with torch.no_grad():
        if with_decay:
            w.mul_(1.0 - lr * lr_ratio * coeff)
        m1.mul_(beta1).add_(g, alpha=1 - beta1)
        m2.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        bc1 = 1 - b1p.float().reshape(-1)[0]
        bc2 = 1 - b2p.float().reshape(-1)[0]
        upd = (m1 / bc1) / ((m2 / bc2).sqrt() + epsilon)
        w.sub_((lr * lr_ratio) * upd.to(w.dtype))
        if master is not None:
            p.copy_(master.to(p.dtype))
        if not use_global_beta_pow:
            b1p.mul_(beta1)
            b2p.mul_(beta2)
    return param, moment1, moment2, None, beta1_pow, beta2_pow, master_param


_ALIASES = {'elementwise_add': 'add', 'elementwise_sub': 'subtract', 'elementwise_mul': 'multiply',
            'elementwise_div': 'divide', 'reduce_sum': 'sum', 'reduce_mean': 'mean', 'matmul_v2': 'matmul',
            'lookup_table_v2': 'embedding', 'fill_constant': 'full'}


def check_finite_and_unscale_(x, scale, found_inf):
    """xs *= 1/scale in place, found_inf set on any inf/nan (csrc/amp.hip, one launch per 48)."""
    from .core.tensor import _unwrap
    from .ops.amp import check_finite_and_unscale_ as _k
    import torch
    xs = [_unwrap(t) for t in x]
    f = _unwrap(found_inf)
    ft = torch.zeros(1, dtype=torch.float32, device=f.device)
    _k(xs, _unwrap(scale).float().reshape(1), ft)
    f.copy_((ft.reshape(f.shape) != 0).to(f.dtype))
    return x, found_inf


def update_loss_scaling_(x, found_inf, prev_loss_scaling, in_good_steps, in_bad_steps, incr_every_n_steps,
                         decr_every_n_nan_or_inf, incr_ratio, decr_ratio, stop_update=False):
    """Dynamic loss-scale update on device scalars; gradients zeroed when found_inf (reference
    update_loss_scaling op semantics)."""
    from .core.tensor import _unwrap
    from .ops.amp import update_loss_scaling_ as _k
    import torch
    f = _unwrap(found_inf)
    ff = f.float().reshape(1)
    bad = ff != 0  # device bool, no host sync
    for t in x:
        tt = _unwrap(t)
        # assign zeros (reference FusedFillIf, phi/kernels/gpu/amp_kernel.cu:212): a gradient
        # holding inf / nan would stay nan under a multiply by 0
        tt.masked_fill_(bad.reshape([1] * tt.dim()) if tt.dim() else bad.reshape(()), 0)
    if stop_update:
        return x, prev_loss_scaling, in_good_steps, in_bad_steps
    sc, g, b = _unwrap(prev_loss_scaling), _unwrap(in_good_steps), _unwrap(in_bad_steps)
    s32, g32, b32 = sc.float().reshape(1).clone(), g.float().reshape(1).clone(), b.float().reshape(1).clone()
    _k(ff, s32, g32, b32, incr_every_n_steps, decr_every_n_nan_or_inf, incr_ratio, decr_ratio)
    sc.copy_(s32.reshape(sc.shape).to(sc.dtype))
    g.copy_(g32.reshape(g.shape).to(g.dtype))
    b.copy_(b32.reshape(b.shape).to(b.dtype))
    return x, prev_loss_scaling, in_good_steps, in_bad_steps


def _inplace_of(fn, name):
    """An in-place ``name`` built from its out-of-place op: the result is written back into the
    first argument's storage (same shape and dtype required), which is returned."""
    def f(x, *a, **k):
        from .core.tensor import _unwrap
        out = fn(x, *a, **k)
        xt, ot = _unwrap(x), _unwrap(out)
        if tuple(ot.shape) != tuple(xt.shape):
            raise ValueError(f"paddle._C_ops.{name}: result shape {tuple(ot.shape)} != input {tuple(xt.shape)}")
        xt.copy_(ot.to(xt.dtype))
        return x
    f.__name__ = name
    return f


def __getattr__(name):
    if name in _ALIASES:
        return globals()[_ALIASES[name]]
    inplace = name.endswith('_') and not name.endswith('__')
    base = name[:-1] if inplace else name
    for mod in (_P(), _F()):
        fn = getattr(mod, name, None)
        if callable(fn):
            return fn
    if inplace:  # no in-place function: keep the in-place contract explicitly
        for mod in (_P(), _F()):
            fn = getattr(mod, base, None)
            if callable(fn):
                return _inplace_of(fn, name)
    raise AttributeError(f"paddle._C_ops has no operator '{name}'")
