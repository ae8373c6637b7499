"""paddle.nn.functional normalisation (reference: python/paddle/nn/functional/norm.py,
python/paddle/incubate/nn/functional/{fused_rms_norm,fused_layer_norm}.py).

layer_norm / rms_norm over the last dim of a HIP tensor run the hand-written
``csrc/norm.hip`` kernels (one wave per row, bf16 vectorised, fp32 statistics).
"""
import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ... import ops
from ...core.amp_dispatch import amp_op as _amp_op


@_amp_op('layer_norm')
def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-05, name=None):
    t = _u(x)
    if isinstance(normalized_shape, int):
        normalized_shape = [normalized_shape]
    ns = list(normalized_shape)
    w = _u(weight) if weight is not None else None
    b = _u(bias) if bias is not None else None
    if ops.use_hip(t) and len(ns) == 1 and w is not None and b is not None:
        return _w(ops.norm.layer_norm(t, w, b, epsilon))
    return _w(TF.layer_norm(t, ns, w, b, epsilon))


def rms_norm(x, normalized_shape, weight=None, epsilon=1e-05, name=None):
    t = _u(x)
    w = _u(weight) if weight is not None else None
    if ops.use_hip(t) and w is not None:
        return _w(ops.norm.rms_norm(t, w, epsilon))
    tf = t.float() if t.dtype in (torch.float16, torch.bfloat16) else t
    var = tf.pow(2).mean(-1, keepdim=True)
    y = (tf * torch.rsqrt(var + epsilon)).to(t.dtype)
    # output in the input's dtype (an fp32 weight under AMP-O2 must not promote a bf16 activation,
    # matching the HIP kernel path)
    return _w(y * w.to(t.dtype) if w is not None else y)


def batch_norm(x, running_mean, running_var, weight=None, bias=None, training=False, momentum=0.9, epsilon=1e-05,
               data_format='NCHW', use_global_stats=None, name=None):
    t = _u(x)
    cl = data_format[-1] == 'C' and t.dim() > 2
    use_batch = training if use_global_stats is None else not use_global_stats
    rm, rv = _u(running_mean), _u(running_var)
    g = None if weight is None else _u(weight)
    if cl and use_batch and ops.use_hip(t) and ops.batchnorm.supported(t, g):
        # channels-last activation = [rows, C] matrix: column-blocked HIP statistics + apply kernels
        return _w(ops.batchnorm.bn_act_nhwc(t, g, None if bias is None else _u(bias), rm, rv, epsilon, momentum,
                                            True))
    if not cl and t.dim() == 4 and ops.use_hip(t) and t.is_contiguous(memory_format=torch.channels_last) \
            and ops.batchnorm.supported(t.permute(0, 2, 3, 1), g) \
            and (use_batch or not (torch.is_grad_enabled() and any(
                v is not None and v.requires_grad for v in (t, g, None if bias is None else _u(bias))))):
        # NCHW view with channels-last strides (a routed conv2d output): the same kernels on the
        # NHWC image (inference with running statistics included: no backward needed there)
        y = ops.batchnorm.bn_act_nhwc(t.permute(0, 2, 3, 1), g, None if bias is None else _u(bias), rm, rv, epsilon,
                                      momentum, bool(use_batch))
        return _w(y.permute(0, 3, 1, 2))
    if use_batch and ops.use_hip(t) and t.dim() == 4 and (cl or t.is_contiguous(memory_format=torch.channels_last)) \
            and ops.batchnorm.channel_pad_ok(t, g):
        # channel count off the kernels' 16-byte grain (ShuffleNetV2 58/116/232): zero-padded copy
        b = None if bias is None else _u(bias)
        if cl:
            return _w(ops.batchnorm.bn_nhwc_cpad(t, g, b, rm, rv, epsilon, momentum, True))
        y = ops.batchnorm.bn_nhwc_cpad(t.permute(0, 2, 3, 1), g, b, rm, rv, epsilon, momentum, True)
        return _w(y.permute(0, 3, 1, 2))
    if cl:
        t = t.permute(0, t.dim() - 1, *range(1, t.dim() - 1))
    out = TF.batch_norm(t, rm, rv, None if weight is None else _u(weight), None if bias is None else _u(bias),
                        use_batch, 1.0 - momentum, epsilon)
    if cl:
        out = out.permute(0, *range(2, out.dim()), 1)
    return _w(out)


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats=True, momentum=0.9,
                  eps=1e-05, data_format='NCHW', name=None):
    t = _u(x)
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, t.dim() - 1, *range(1, t.dim() - 1))
    out = TF.instance_norm(t, _u(running_mean), _u(running_var), _u(weight), _u(bias), use_input_stats,
                           1.0 - momentum, eps)
    if cl:
        out = out.permute(0, *range(2, out.dim()), 1)
    return _w(out)


@_amp_op('group_norm')
def group_norm(x, num_groups, epsilon=1e-05, weight=None, bias=None, data_format='NCHW', name=None):
    t = _u(x)
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, t.dim() - 1, *range(1, t.dim() - 1))
    out = TF.group_norm(t, num_groups, _u(weight), _u(bias), epsilon)
    if cl:
        out = out.permute(0, *range(2, out.dim()), 1)
    return _w(out)


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0, data_format='NCHW', name=None):
    t = _u(x)
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, t.dim() - 1, *range(1, t.dim() - 1))
    out = TF.local_response_norm(t, size, alpha, beta, k)
    if cl:
        out = out.permute(0, *range(2, out.dim()), 1)
    return _w(out)
