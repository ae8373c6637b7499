"""Strided-row RoPE kernel (pa_rope_rows) and the fused QKV -> RoPE -> flash attention op
(ops.flash_attn.qkv_rope_flash, the Llama attention path) vs fp32 torch references."""
import math

import pytest
import torch

import paddle  # noqa: F401
from paddle.ops import rope, flash_attn as FA

pytestmark = pytest.mark.gpu


def _rope_ref(x, cos, sin, pos, interleaved):
    """x [B, S, H, D] fp32; cos/sin [S_max, D/2]."""
    B, S, H, D = x.shape
    p = pos if pos is not None else torch.arange(S, device=x.device)[None].expand(B, S)
    c, s = cos[p][:, :, None, :], sin[p][:, :, None, :]
    if interleaved:
        a, b = x[..., 0::2], x[..., 1::2]
        return torch.stack([a * c - b * s, b * c + a * s], -1).reshape(B, S, H, D)
    a, b = x[..., :D // 2], x[..., D // 2:]
    return torch.cat([a * c - b * s, b * c + a * s], -1)


@pytest.mark.parametrize('interleaved', [False, True])
@pytest.mark.parametrize('use_pos', [False, True])
def test_rope_rows_strided_and_inplace(interleaved, use_pos):
    torch.manual_seed(0)
    B, S, H, D = 2, 96, 12, 128
    qkv = torch.randn(B, S, 3 * H, D, device='cuda').bfloat16()
    cos, sin = rope.rope_tables(256, D, 10000.0, 'cuda')
    pos = torch.randint(0, 256, (B, S), device='cuda') if use_pos else None
    x = qkv[:, :, H:2 * H]                      # strided slice
    assert rope.rows_ok(x)
    y = torch.empty(B, S, H, D, device='cuda').bfloat16()
    rope.rope_rows(x, y, cos, sin, pos, interleaved)
    ref = _rope_ref(x.float(), cos, sin, pos, interleaved)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=1e-2)
    z = qkv.clone()
    zs = z[:, :, H:2 * H]
    rope.rope_rows(zs, zs, cos, sin, pos, interleaved)           # in place
    torch.testing.assert_close(zs.float(), y.float(), atol=0, rtol=0)
    torch.testing.assert_close(z[:, :, :H], qkv[:, :, :H], atol=0, rtol=0)  # neighbours untouched
    rope.rope_rows(zs, zs, cos, sin, pos, interleaved, sign=-1.0)            # inverse rotation
    torch.testing.assert_close(zs.float(), x.float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize('nh,nkv', [(8, 8), (8, 2)])
@pytest.mark.parametrize('use_pos', [False, True])
def test_qkv_rope_flash_matches_reference(nh, nkv, use_pos):
    torch.manual_seed(1)
    B, S, D = 2, 256, 128
    cos, sin = rope.rope_tables(512, D, 10000.0, 'cuda')
    pos = torch.arange(S, device='cuda')[None].expand(B, S).contiguous() + 7 if use_pos else None
    qkv = (torch.randn(B, S, nh + 2 * nkv, D, device='cuda') * 0.5).bfloat16().requires_grad_()
    assert FA.qkv_rope_flash_ok(qkv, nh, nkv)
    o = FA.qkv_rope_flash(qkv, nh, nkv, cos, sin, pos, causal=True)
    g = torch.randn_like(o)
    o.backward(g)
    # fp32 reference
    qr = qkv.detach().float().requires_grad_()
    q = _rope_ref(qr[:, :, :nh], cos, sin, pos, False)
    k = _rope_ref(qr[:, :, nh:nh + nkv], cos, sin, pos, False)
    v = qr[:, :, nh + nkv:]
    k = k.repeat_interleave(nh // nkv, 2)
    v = v.repeat_interleave(nh // nkv, 2)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(D)
    s = s.masked_fill(torch.ones(S, S, device='cuda', dtype=torch.bool).triu(1), float('-inf'))
    ref = torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v)
    ref.backward(g.float())
    torch.testing.assert_close(o.float(), ref, atol=3e-2, rtol=2e-2)
    err = (qkv.grad.float() - qr.grad).abs().max().item() / qr.grad.abs().max().item()
    assert err < 3e-2, err


def test_swiglu_packed_single_gradient_buffer():
    """F.swiglu(x) of the fused gate/up projection: one packed autograd op (no chunk / cat), values
    and the gradient vs fp32 torch."""
    import paddle.nn.functional as F
    torch.manual_seed(2)
    x = torch.randn(3, 50, 2 * 1024, device='cuda').bfloat16().requires_grad_()
    xp = paddle.to_tensor(x.detach(), stop_gradient=False)
    yp = F.swiglu(xp)
    g = torch.randn(3, 50, 1024, device='cuda')
    yp.backward(paddle.to_tensor(g.bfloat16()))
    xr = x.detach().float().requires_grad_()
    a, b = xr.chunk(2, -1)
    ref = torch.nn.functional.silu(a) * b
    ref.backward(g)
    torch.testing.assert_close(yp._t.float(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(xp.grad._t.float(), xr.grad, atol=5e-2, rtol=3e-2)
