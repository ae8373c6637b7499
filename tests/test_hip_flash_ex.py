"""GPU numerics of the extended flash-attention kernels (csrc/flash_attn.hip *_ex entry points):
additive / bool masks, in-kernel dropout, varlen (cu_seqlens) packing, padded head dims —
forward and backward against a plain fp32 PyTorch reference of the same op.

Reference behaviour: python/paddle/nn/functional/flash_attention.py (flash_attention dropout,
flash_attn_unpadded, scaled_dot_product_attention attn_mask, flashmask startend_row_indices).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

DEV = 'cuda'
FA = ops.flash_attn


def setup_module(m):
    torch.manual_seed(0)
    assert _native._load() is not None, _native.load_error


def _close(a, b, atol, rtol=0.0, name=''):
    a, b = a.float(), b.float()
    assert torch.isfinite(a).all(), f"{name}: non-finite values"
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{name}: max err {err} > {tol}"


def _ref(q, k, v, causal, mask=None, z=None, scale=None):
    """fp32 attention on [B, S, H, D]; mask additive/bool broadcastable to [B, H, Sq, Sk]; z the
    dropout keep-scale [B, H, Sq, Sk] applied to the normalised probabilities."""
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if kf.shape[1] != qf.shape[1]:
        rep = qf.shape[1] // kf.shape[1]
        kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    s = qf @ kf.transpose(-1, -2) * (scale if scale is not None else 1 / math.sqrt(q.shape[-1]))
    if mask is not None:
        s = s.masked_fill(~mask, float('-inf')) if mask.dtype == torch.bool else s + mask.float()
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1 + Sk - Sq), float('-inf'))
    p = torch.softmax(s, -1)
    p = torch.nan_to_num(p, nan=0.0)
    if z is not None:
        p = p * z
    return (p @ vf).transpose(1, 2)


def _leaf(*shape, dt=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dt).requires_grad_()


def _grads_vs_ref(out, ref, ins, ref_ins, tol, name):
    g = torch.randn_like(ref)
    out.backward(g.to(out.dtype))
    ref.backward(g)
    for a, b, n in zip(ins, ref_ins, 'qkv'):
        _close(a.grad, b.grad, tol, 2e-2, f'{name} d{n}')


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("kind", ['f32', 'bf16', 'bool'])
def test_flash_mask(D, causal, kind):
    B, Sq, Sk, H = 2, 200, 264, 4
    q, k, v = _leaf(B, Sq, H, D), _leaf(B, Sk, H, D), _leaf(B, Sk, H, D)
    if kind == 'bool':
        mask = torch.rand(B, H, Sq, Sk, device=DEV) > 0.3
        mask[..., -1] = True  # no fully masked row (its reference row is NaN)
    else:
        mask = torch.randn(B, 1, Sq, Sk, device=DEV) * 2
        mask[:, :, :, 5:40] = float('-inf')
        mask = mask.to(torch.float32 if kind == 'f32' else torch.bfloat16)
    o = FA.flash_attention_ex(q, k, v, causal, mask=mask)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal, mask=mask)
    _close(o, r, 2e-2, name=f'mask {kind} fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, f'mask {kind}')


def test_flash_fully_masked_rows_are_zero():
    B, S, H, D = 1, 128, 2, 64
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    mask = torch.ones(B, 1, S, S, dtype=torch.bool, device=DEV)
    mask[:, :, 10] = False
    o = FA.flash_attention_ex(q, k, v, False, mask=mask)
    assert o[:, 10].abs().max().item() == 0
    o.sum().backward()
    for t in (q, k, v):
        assert torch.isfinite(t.grad).all()
    assert q.grad[:, 10].abs().max().item() == 0


def _dropout_mask(B, S, H, D, causal, p, seed):
    """Recover the kernel's keep mask: with V = one-hot keys (Sk = D) row q of O is P[q]·Z[q]."""
    q = (torch.randn(B, S, H, D, device=DEV) * 0.3).bfloat16()
    k = (torch.randn(B, S, H, D, device=DEV) * 0.3).bfloat16()
    v = torch.eye(S, D, device=DEV).bfloat16().view(1, S, 1, D).expand(B, S, H, D).contiguous()
    torch.manual_seed(seed)
    o = FA.flash_attention_ex(q, k, v, causal, dropout=p)
    z = (o.float().transpose(1, 2)[..., :S] > 0).float() / (1 - p)  # [B, H, Sq, Sk]
    return q, k, v, o, z


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [64, 128])
def test_flash_dropout(causal, D):
    B, S, H, p = 2, D, 3, 0.25
    q, k, v, o, z = _dropout_mask(B, S, H, D, causal, p, seed=123)
    allowed = torch.ones(S, S, device=DEV, dtype=torch.bool)
    if causal:
        allowed = allowed.tril()
    kept = (z[..., allowed] > 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.03, kept
    _close(o, _ref(q, k, v, causal, z=z), 2e-2, name='dropout fwd')
    # same seed → the same mask; gradients against the reference with that mask
    qq, kk, vv = _leaf(B, S, H, D, scale=0.3), _leaf(B, S, H, D, scale=0.3), _leaf(B, S, H, D)
    torch.manual_seed(123)
    o2 = FA.flash_attention_ex(qq, kk, vv, causal, dropout=p)
    ri = [t.detach().float().requires_grad_() for t in (qq, kk, vv)]
    r = _ref(*ri, causal, z=z)
    _close(o2, r, 3e-2, name='dropout fwd2')
    _grads_vs_ref(o2, r, (qq, kk, vv), ri, 6e-2, 'dropout')


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_flash_dropout_statistics(p):
    """Keep mask recovered from the kernel (one-hot V): keep rate, and no correlation between
    neighbouring keys, key quads or queries (the hash must not leak structure into the mask)."""
    B, S, H, D = 1, 128, 8, 128
    _, _, _, _, z = _dropout_mask(B, S, H, D, False, p, seed=7)
    keep = (z > 0).float().reshape(-1, S, S)  # [H, Sq, Sk]
    n = keep.numel()
    assert abs(keep.mean().item() - (1 - p)) < 4 * (p * (1 - p) / n) ** 0.5 + 2 / 256, keep.mean().item()

    def corr(a, b):
        a, b = a.reshape(-1) - a.mean(), b.reshape(-1) - b.mean()
        return (a @ b / (a.norm() * b.norm())).item()
    tol = 5 / (n ** 0.5)
    for name, (a, b) in {'key': (keep[..., :-1], keep[..., 1:]), 'key+4': (keep[..., :-4], keep[..., 4:]),
                         'query': (keep[:, :-1], keep[:, 1:]), 'head': (keep[:-1], keep[1:])}.items():
        assert abs(corr(a, b)) < tol, (name, corr(a, b))


def test_flash_dropout_packed_matches_unpacked():
    B, S, H, D, p = 2, 256, 4, 128, 0.1
    qkv = _leaf(B, S, 3, H, D)
    torch.manual_seed(7)
    o1 = FA.flash_attention_packed_ex(qkv, True, dropout=p)
    o1.sum().backward()
    g1 = qkv.grad.clone()
    qkv.grad = None
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    torch.manual_seed(7)
    o2 = FA.flash_attention_ex(q, k, v, True, dropout=p)
    o2.sum().backward()
    assert torch.equal(o1, o2)
    _close(g1, qkv.grad, 1e-6, name='packed vs views')
    # dropout actually changes the output, but keeps its scale
    o0 = FA.flash_attention_packed(qkv.detach(), True)
    assert (o1 - o0).abs().max().item() > 1e-2


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D,Hq,Hk", [(64, 4, 4), (128, 4, 2)])
def test_flash_varlen(causal, D, Hq, Hk):
    lens_q = [37, 128, 1, 200, 64]
    lens_k = lens_q if causal else [50, 128, 9, 190, 70]
    cq = torch.tensor([0] + lens_q, device=DEV).cumsum(0).int()
    ck = torch.tensor([0] + lens_k, device=DEV).cumsum(0).int()
    q, k, v = _leaf(sum(lens_q), Hq, D), _leaf(sum(lens_k), Hk, D), _leaf(sum(lens_k), Hk, D)
    o = FA.flash_attention_ex(q, k, v, causal, cu_seqlens_q=cq, cu_seqlens_k=ck)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    outs = []
    for i in range(len(lens_q)):
        a, b = cq[i].item(), cq[i + 1].item()
        c, d = ck[i].item(), ck[i + 1].item()
        outs.append(_ref(ri[0][a:b][None], ri[1][c:d][None], ri[2][c:d][None], causal)[0])
    r = torch.cat(outs)
    _close(o, r, 2e-2, name='varlen fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'varlen')


def test_flash_varlen_with_mask_and_dropout_runs():
    lens = [100, 30, 129]
    cu = torch.tensor([0] + lens, device=DEV).cumsum(0).int()
    T, H, D = sum(lens), 2, 64
    q, k, v = _leaf(T, H, D), _leaf(T, H, D), _leaf(T, H, D)
    mask = torch.zeros(len(lens), 1, max(lens), max(lens), device=DEV)
    o = FA.flash_attention_ex(q, k, v, True, mask=mask, cu_seqlens_q=cu, cu_seqlens_k=cu)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = torch.cat([_ref(ri[0][a:b][None], ri[1][a:b][None], ri[2][a:b][None], True)[0]
                   for a, b in zip(cu[:-1].tolist(), cu[1:].tolist())])
    _close(o, r, 2e-2, name='varlen+mask fwd')
    o2 = FA.flash_attention_ex(q, k, v, True, dropout=0.2, cu_seqlens_q=cu, cu_seqlens_k=cu)
    o2.float().sum().backward()
    assert torch.isfinite(q.grad).all()


@pytest.mark.parametrize("D", [32, 80, 96])
def test_flash_padded_head_dim(D):
    B, S, H = 2, 160, 4
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    from paddle.core.tensor import _wrap
    out, _ = paddle.nn.functional.flash_attention(_wrap(q), _wrap(k), _wrap(v), causal=True)
    o = out._t
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, True)
    _close(o, r, 2e-2, name=f'D{D} fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, f'D{D}')


def test_api_routes_mask_and_dropout_to_kernel(monkeypatch):
    """nn.functional with a mask / dropout must run the HIP kernel, not the SDPA fallback."""
    import sys
    M = sys.modules[paddle.nn.functional.flash_attention.__module__]
    called = []
    monkeypatch.setattr(M, '_sdpa_reference', lambda *a, **k: called.append(1))
    B, S, H, D = 2, 128, 4, 64
    x = paddle.to_tensor(torch.randn(B, S, H, D, device=DEV).bfloat16())
    m = paddle.to_tensor(torch.zeros(B, 1, S, S, device=DEV))
    paddle.nn.functional.scaled_dot_product_attention(x, x, x, attn_mask=m)
    paddle.nn.functional.flash_attention(x, x, x, dropout=0.1, causal=True)
    qkv = paddle.to_tensor(torch.randn(B, S, 3, H, D, device=DEV).bfloat16())
    paddle.nn.functional.flash_attn_qkvpacked(qkv, dropout=0.1, causal=True)
    t = paddle.to_tensor(torch.randn(2 * S, H, D, device=DEV).bfloat16())
    cu = paddle.to_tensor(torch.tensor([0, 100, 2 * S], dtype=torch.int32, device=DEV))
    paddle.nn.functional.flash_attn_unpadded(t, t, t, cu, cu, 156, 156, 0.125, causal=True)
    assert not called


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D,Hr", [(64, 4), (128, 1)])
def test_flash_startend_rows(causal, D, Hr):
    """flashmask: key k hidden from query rows >= rows[b, h, k] (h broadcast when Hr == 1)."""
    B, S, H = 2, 300, 4
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    rows = torch.randint(S // 3, S + 1, (B, Hr, S), device=DEV, dtype=torch.int32)
    rows[..., 0] = S  # key 0 visible to every row: no empty softmax row
    o = FA.flash_attention_ex(q, k, v, causal, start_rows=rows)
    keep = torch.arange(S, device=DEV).view(1, 1, S, 1) < rows.unsqueeze(2)  # [B, Hr, Sq, Sk]
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal, mask=keep)
    _close(o, r, 2e-2, name='flashmask fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'flashmask')


def test_sparse_mask_api_matches_dense():
    B, S, H, D = 1, 256, 2, 64
    x = torch.randn(B, S, H, D, device=DEV).bfloat16()
    rows = torch.randint(S // 2, S + 1, (B, H, S), device=DEV, dtype=torch.int32)
    out = paddle.nn.functional.flash_attention_with_sparse_mask(
        paddle.to_tensor(x), paddle.to_tensor(x), paddle.to_tensor(x), paddle.to_tensor(rows), is_causal=True)
    keep = torch.arange(S, device=DEV).view(1, 1, S, 1) < rows.unsqueeze(2)
    _close(out._t, _ref(x, x, x, True, mask=keep), 2e-2, name='sparse api')
