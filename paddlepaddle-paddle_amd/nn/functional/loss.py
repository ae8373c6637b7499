"""paddle.nn.functional losses (reference: python/paddle/nn/functional/loss.py).

Hard-label cross_entropy on a HIP tensor uses the fused softmax-cross-entropy kernel
(``csrc/xent.hip``): one pass computes the row logsumexp and the loss, backward writes
softmax − onehot in place of a materialised probability tensor.
"""
import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ... import ops
from ...core.amp_dispatch import amp_op as _amp_op


def _reduce(t, reduction):
    if reduction == 'mean':
        return t.mean()
    if reduction == 'sum':
        return t.sum()
    return t


def _acc(t):
    """Accumulation dtype of a loss: float32 for half types, the input's own dtype otherwise."""
    return t.float() if t.dtype in (torch.float16, torch.bfloat16) else t


@_amp_op('cross_entropy')
def cross_entropy(input, label, weight=None, ignore_index=-100, reduction='mean', soft_label=False, axis=-1,  # noqa: A002
                  use_softmax=True, label_smoothing=0.0, name=None):
    logits, lab = _u(input), _u(label)
    axis = axis % logits.dim()
    w = _u(weight) if weight is not None else None
    if soft_label or (lab.is_floating_point() and lab.shape == logits.shape):
        lf = _acc(logits)
        logp = torch.log_softmax(lf, axis) if use_softmax else torch.log(lf)
        if label_smoothing:
            lab = lab * (1 - label_smoothing) + label_smoothing / logits.shape[axis]
        loss = -(lab * logp)
        if w is not None:
            shape = [1] * logits.dim()
            shape[axis] = -1
            loss = loss * w.reshape(shape)
        loss = loss.sum(axis, keepdim=True).to(logits.dtype)
        if reduction == 'none':
            return _w(loss)
        return _w(_reduce(loss, reduction))
    if lab.dim() == logits.dim() and lab.shape[axis] == 1:
        lab = lab.squeeze(axis)
    lab = lab.long()
    if (use_softmax and w is None and label_smoothing == 0.0 and axis == logits.dim() - 1 and ops.use_hip(logits)):
        loss = ops.xent.softmax_cross_entropy(logits.reshape(-1, logits.shape[-1]), lab.reshape(-1), ignore_index)
        loss = loss.reshape(lab.shape)
        if reduction == 'none':
            return _w(loss.unsqueeze(-1).to(logits.dtype))
        if reduction == 'sum':
            return _w(loss.sum())
        valid = (lab != ignore_index).sum().clamp_min(1)
        return _w(loss.sum() / valid)
    if axis != logits.dim() - 1:
        logits = logits.movedim(axis, -1)
    lg = logits.reshape(-1, logits.shape[-1])
    if not use_softmax:
        lg = torch.log(lg)
        lg = _acc(lg)
        loss = TF.nll_loss(lg, lab.reshape(-1), None if w is None else w.to(lg.dtype), ignore_index=ignore_index,
                           reduction='none')
    else:
        lg = _acc(lg)
        loss = TF.cross_entropy(lg, lab.reshape(-1), None if w is None else w.to(lg.dtype), ignore_index=ignore_index,
                                reduction='none',
                                label_smoothing=label_smoothing)
    loss = loss.reshape(lab.shape)
    if reduction == 'none':  # label-shaped: the class axis kept as a unit dim at `axis`
        return _w(loss.unsqueeze(axis).to(logits.dtype))
    out_dt = logits.dtype if logits.dtype in (torch.float32, torch.float64) else loss.dtype
    if reduction == 'sum':
        return _w(loss.sum().to(out_dt))
    if w is not None:
        wsum = w.to(loss.dtype)[lab.clamp_min(0)].masked_fill(lab == ignore_index, 0).sum()
        return _w((loss.sum() / wsum).to(out_dt))
    valid = (lab != ignore_index).sum().clamp_min(1)
    return _w((loss.sum() / valid).to(out_dt))


@_amp_op('softmax_with_cross_entropy')
def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=True,
                               return_softmax=False, axis=-1):
    loss = cross_entropy(logits, label, soft_label=soft_label, ignore_index=ignore_index, reduction='none', axis=axis)
    if return_softmax:
        return loss, _w(torch.softmax(_u(logits), axis))
    return loss


@_amp_op('nll_loss')
def nll_loss(input, label, weight=None, ignore_index=-100, reduction='mean', name=None):  # noqa: A002
    t, l = _u(input), _u(label).long()
    if t.dim() > 2:
        return _w(TF.nll_loss(t, l, _u(weight), ignore_index=ignore_index, reduction=reduction))
    return _w(TF.nll_loss(t, l, _u(weight), ignore_index=ignore_index, reduction=reduction))


def mse_loss(input, label, reduction='mean', name=None):  # noqa: A002
    return _w(TF.mse_loss(_u(input), _u(label), reduction=reduction))


def square_error_cost(input, label):  # noqa: A002
    return _w((_u(input) - _u(label)) ** 2)


def l1_loss(input, label, reduction='mean', name=None):  # noqa: A002
    return _w(TF.l1_loss(_u(input), _u(label), reduction=reduction))


@_amp_op('huber_loss')
def smooth_l1_loss(input, label, reduction='mean', delta=1.0, name=None):  # noqa: A002
    return _w(TF.huber_loss(_u(input), _u(label), reduction=reduction, delta=delta))


def binary_cross_entropy(input, label, weight=None, reduction='mean', name=None):  # noqa: A002
    return _w(TF.binary_cross_entropy(_u(input), _u(label), _u(weight), reduction=reduction))


@_amp_op('sigmoid_cross_entropy_with_logits')
def binary_cross_entropy_with_logits(logit, label, weight=None, reduction='mean', pos_weight=None, name=None):
    return _w(TF.binary_cross_entropy_with_logits(_u(logit), _u(label), _u(weight), reduction=reduction,
                                                  pos_weight=_u(pos_weight)))


def sigmoid_focal_loss(logit, label, normalizer=None, alpha=0.25, gamma=2.0, reduction='sum', name=None):
    x, y = _u(logit), _u(label)
    p = torch.sigmoid(x)
    ce = TF.binary_cross_entropy_with_logits(x, y, reduction='none')
    pt = p * y + (1 - p) * (1 - y)
    loss = ce * (1 - pt) ** gamma
    if alpha >= 0:
        loss = (alpha * y + (1 - alpha) * (1 - y)) * loss
    if normalizer is not None:
        loss = loss / _u(normalizer)
    return _w(_reduce(loss, reduction))


def kl_div(input, label, reduction='mean', log_target=False, name=None):  # noqa: A002
    t, l = _u(input), _u(label)
    loss = torch.exp(l) * (l - t) if log_target else l * (torch.log(l.clamp_min(1e-30)) - t)
    loss = torch.where(l > 0, loss, torch.zeros_like(loss)) if not log_target else loss
    if reduction == 'batchmean':
        return _w(loss.sum() / t.shape[0])
    return _w(_reduce(loss, reduction))


def margin_ranking_loss(input, other, label, margin=0.0, reduction='mean', name=None):  # noqa: A002
    return _w(TF.margin_ranking_loss(_u(input), _u(other), _u(label), margin=margin, reduction=reduction))


def hinge_embedding_loss(input, label, margin=1.0, reduction='mean', name=None):  # noqa: A002
    return _w(TF.hinge_embedding_loss(_u(input), _u(label), margin=margin, reduction=reduction))


def cosine_embedding_loss(input1, input2, label, margin=0, reduction='mean', name=None):
    return _w(TF.cosine_embedding_loss(_u(input1), _u(input2), _u(label), margin=margin, reduction=reduction))


@_amp_op('triplet_margin_loss')
def triplet_margin_loss(input, positive, negative, margin=1.0, p=2, epsilon=1e-6, swap=False, reduction='mean',  # noqa: A002
                        name=None):
    return _w(TF.triplet_margin_loss(_u(input), _u(positive), _u(negative), margin=margin, p=p, eps=epsilon,
                                     swap=swap, reduction=reduction))


def triplet_margin_with_distance_loss(input, positive, negative, distance_function=None, margin=1.0, swap=False,  # noqa: A002
                                      reduction='mean', name=None):
    df = None
    if distance_function is not None:
        df = lambda a, b: _u(distance_function(_w(a), _w(b)))  # noqa: E731
    return _w(TF.triplet_margin_with_distance_loss(_u(input), _u(positive), _u(negative), distance_function=df,
                                                   margin=margin, swap=swap, reduction=reduction))


def multi_label_soft_margin_loss(input, label, weight=None, reduction='mean', name=None):  # noqa: A002
    return _w(TF.multilabel_soft_margin_loss(_u(input), _u(label), _u(weight), reduction=reduction))


def multi_margin_loss(input, label, p=1, margin=1.0, weight=None, reduction='mean', name=None):  # noqa: A002
    return _w(TF.multi_margin_loss(_u(input), _u(label).long(), p, margin, _u(weight), reduction=reduction))


def soft_margin_loss(input, label, reduction='mean', name=None):  # noqa: A002
    return _w(TF.soft_margin_loss(_u(input), _u(label), reduction=reduction))


def poisson_nll_loss(input, label, log_input=True, full=False, epsilon=1e-8, reduction='mean', name=None):  # noqa: A002
    return _w(TF.poisson_nll_loss(_u(input), _u(label), log_input, full, eps=epsilon, reduction=reduction))


def gaussian_nll_loss(input, label, variance, full=False, epsilon=1e-6, reduction='mean', name=None):  # noqa: A002
    return _w(TF.gaussian_nll_loss(_u(input), _u(label), _u(variance), full, epsilon, reduction))


@_amp_op('log_loss')
def log_loss(input, label, epsilon=1e-4, name=None):  # noqa: A002
    x, y = _u(input), _u(label)
    return _w(-y * torch.log(x + epsilon) - (1 - y) * torch.log(1 - x + epsilon))


def dice_loss(input, label, epsilon=0.00001, name=None):  # noqa: A002
    x, y = _u(input), _u(label)
    y = TF.one_hot(y.squeeze(-1).long(), x.shape[-1]).to(x.dtype)
    dims = tuple(range(1, x.dim()))
    inse = (x * y).sum(dims)
    return _w((1 - 2 * inse / (x.sum(dims) + y.sum(dims) + epsilon)).mean())


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    a, p, l = _u(anchor), _u(positive), _u(labels).reshape(-1, 1).float()
    reg = l2_reg * ((a ** 2).sum(1).mean() + (p ** 2).sum(1).mean()) * 0.25
    sim = (l == l.t()).float()
    sim = sim / sim.sum(1, keepdim=True)
    logits = a @ p.t()
    ce = (-sim * torch.log_softmax(logits, 1)).sum(1).mean()
    return _w(ce + reg)


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction='mean', norm_by_times=False):
    lp = _u(log_probs)
    loss = TF.ctc_loss(lp.log_softmax(-1) if lp.max() > 0 else lp, _u(labels), _u(input_lengths), _u(label_lengths),
                       blank, reduction='none')
    if reduction == 'mean':
        return _w((loss / _u(label_lengths).clamp_min(1)).mean())
    return _w(_reduce(loss, reduction))


def rnnt_loss(input, label, input_lengths, label_lengths, blank=0, fastemit_lambda=0.001, reduction='mean', name=None):  # noqa: A002
    """RNN-Transducer loss (reference nn/functional/loss.py:1983 rnnt_loss -> the warprnnt op).

    ``input``: log-probabilities [B, Tmax, Umax+1, V] (used as given, like the reference kernel);
    ``label`` [B, Umax]; per-sequence lengths.  loss_b = -log sum over alignments of the summed
    log-probabilities.  Forward variable alpha is vectorised over (B, U) per time step:
        alpha[t, u] = C[t, u] + logcumsumexp_u'<=u(alpha[t-1, u'] + blank[t-1, u'] - C[t, u'])
    with C[t, u] = sum_{k<u} emit[t, k] (emission of label k at frame t); gradients by autograd.
    FastEmit (arXiv 2010.11148): the label-emission gradients are scaled by (1 + lambda), the value
    is unchanged (the warp-transducer rule).  reduction 'mean' divides the summed loss by B.
    """
    lp = _u(input)
    B, T, U1, V = lp.shape
    lab = _u(label).long().reshape(B, -1)[:, :U1 - 1].clamp(0, V - 1)
    tl = _u(input_lengths).long().reshape(B).to(lp.device) if isinstance(input_lengths, Tensor) else \
        torch.as_tensor(input_lengths, device=lp.device).long().reshape(B)
    ul = _u(label_lengths).long().reshape(B).to(lp.device) if isinstance(label_lengths, Tensor) else \
        torch.as_tensor(label_lengths, device=lp.device).long().reshape(B)
    blank_lp = lp[..., blank]  # [B, T, U1]
    if U1 > 1:
        emit = torch.gather(lp[:, :, :U1 - 1, :], 3, lab[:, None, :, None].expand(B, T, U1 - 1, 1)).squeeze(3)
        if fastemit_lambda:
            emit = emit * (1.0 + fastemit_lambda) - fastemit_lambda * emit.detach()
        C = torch.cat([torch.zeros(B, T, 1, dtype=lp.dtype, device=lp.device), torch.cumsum(emit, 2)], 2)
    else:
        C = torch.zeros(B, T, 1, dtype=lp.dtype, device=lp.device)
    alpha = C[:, 0]
    alphas = [alpha]
    for t in range(1, T):
        a_prev = alpha + blank_lp[:, t - 1]
        alpha = C[:, t] + torch.logcumsumexp(a_prev - C[:, t], 1)
        alphas.append(alpha)
    A = torch.stack(alphas, 1)  # [B, T, U1]
    bi = torch.arange(B, device=lp.device)
    ll = A[bi, tl - 1, ul] + blank_lp[bi, tl - 1, ul]
    loss = -ll
    if reduction == 'mean':
        return _w(loss.sum() / B)
    if reduction == 'sum':
        return _w(loss.sum())
    return _w(loss)


@_amp_op('margin_cross_entropy')
def margin_cross_entropy(logits, label, margin1=1.0, margin2=0.5, margin3=0.0, scale=64.0, group=None,
                         return_softmax=False, reduction='mean'):
    x, y = _u(logits), _u(label).reshape(-1).long()
    theta = torch.acos(x.clamp(-1 + 1e-7, 1 - 1e-7))
    tgt = torch.cos(margin1 * theta + margin2) - margin3
    onehot = TF.one_hot(y, x.shape[-1]).bool()
    z = torch.where(onehot, tgt, x) * scale
    loss = TF.cross_entropy(z, y, reduction='none').unsqueeze(-1)
    loss = _w(_reduce(loss, reduction) if reduction != 'none' else loss)
    if return_softmax:
        return loss, _w(torch.softmax(z, -1))
    return loss


@_amp_op('hsigmoid_loss')
def hsigmoid_loss(input, label, num_classes, weight, bias=None, path_table=None, path_code=None, is_sparse=False,  # noqa: A002
                  name=None):
    x, y, w = _u(input), _u(label).reshape(-1).long(), _u(weight)
    # default complete-binary-tree coding (reference: phi/kernels/funcs/matrix_bit_code.h)
    code_len = max(int(num_classes - 1).bit_length(), 1)
    losses = []
    for i in range(x.shape[0]):
        c = int(y[i]) + num_classes
        l = x.new_zeros(())
        for _ in range(code_len):
            if c <= 1:
                break
            node = c // 2 - 1
            bit = c & 1
            z = (x[i] * w[node]).sum() + (0 if bias is None else _u(bias).reshape(-1)[node])
            l = l + TF.binary_cross_entropy_with_logits(z, torch.tensor(float(bit), device=x.device))
            c //= 2
        losses.append(l)
    return _w(torch.stack(losses).unsqueeze(-1))


def adaptive_log_softmax_with_loss(input, label, head_weight, tail_weights, cutoffs, head_bias=None, name=None):  # noqa: A002
    """Adaptive softmax (reference nn/functional/loss.py:4289): the head scores the shortlist
    [0, cutoffs[0]) plus one logit per tail cluster; a target in cluster i adds the cluster's
    own log-softmax (two projections tail_weights[i-1] = (W_proj [in, hsz], W_out [hsz, osz])).
    Returns (output = log p(label) per row, loss = -mean(output))."""
    x, y = _u(input), _u(label).long()
    batched = y.dim() > 0
    if not batched:
        x, y = x.unsqueeze(0), y.unsqueeze(0)
    if x.dim() != 2 or x.shape[0] != y.shape[0]:
        raise ValueError("input must be [N, in_features] with one label per row")
    cutoffs = list(cutoffs)
    head = x @ _u(head_weight)
    if head_bias is not None:
        head = head + _u(head_bias)
    head_lp = torch.log_softmax(head.float() if head.dtype in (torch.float16, torch.bfloat16) else head, -1)
    short = cutoffs[0]
    out = torch.zeros(x.shape[0], dtype=head_lp.dtype, device=x.device)
    in_short = y < short
    out = torch.where(in_short, head_lp.gather(1, y.clamp(max=short - 1).unsqueeze(1)).squeeze(1), out)
    bounds = cutoffs + ([] if len(tail_weights) + 1 == len(cutoffs) else [])
    for i in range(1, len(cutoffs)):
        lo, hi = cutoffs[i - 1], cutoffs[i]
        m = (y >= lo) & (y < hi)
        if not bool(m.any()):
            continue
        w0, w1 = tail_weights[i - 1]
        logits = (x[m] @ _u(w0)) @ _u(w1)
        lp = torch.log_softmax(logits.to(head_lp.dtype), -1)
        val = head_lp[m, short + i - 1] + lp.gather(1, (y[m] - lo).unsqueeze(1)).squeeze(1)
        out = out.masked_scatter(m, val) if False else out.index_put((m.nonzero().squeeze(1),), val)
    del bounds
    out = out.to(x.dtype)
    if not batched:
        out = out.squeeze(0)
    return _w(out), _w(-out.mean())