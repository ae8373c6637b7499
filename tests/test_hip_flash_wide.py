"""Native head_dim 96 / 256 flash attention (csrc/flash_attn_wide.hip): forward + backward of every
feature (plain, GQA, additive mask, dropout, varlen, flashmask rows) against the fp32 PyTorch
reference, and the paddle API reaching the kernel (no zero padding, no S^2 composite)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

from test_hip_flash_ex import _close, _ref, _leaf, _grads_vs_ref, _dropout_mask  # noqa: E402

DEV = 'cuda'
FA = ops.flash_attn


def setup_module(m):
    torch.manual_seed(0)
    assert _native._load() is not None, _native.load_error


@pytest.mark.parametrize('D', [96, 256])
@pytest.mark.parametrize('causal', [False, True])
@pytest.mark.parametrize('S', [128, 200, 1024])
@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
def test_wide_fwd_bwd(D, causal, S, dt):
    B, H = 2, 2
    q, k, v = _leaf(B, S, H, D, dt=dt), _leaf(B, S, H, D, dt=dt), _leaf(B, S, H, D, dt=dt)
    o = FA.flash_attention(q, k, v, causal)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal)
    _close(o, r, 2e-2, name=f'D{D} fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, f'D{D}')


@pytest.mark.parametrize('D', [96, 256])
def test_wide_gqa_cross_lengths(D):
    B, Sq, Sk, Hq, Hk = 2, 150, 333, 4, 2
    q, k, v = _leaf(B, Sq, Hq, D), _leaf(B, Sk, Hk, D), _leaf(B, Sk, Hk, D)
    for causal in (False, True):
        for t in (q, k, v):
            t.grad = None
        o = FA.flash_attention(q, k, v, causal)
        ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
        r = _ref(*ri, causal)
        _close(o, r, 2e-2, name=f'gqa D{D} fwd')
        _grads_vs_ref(o, r, (q, k, v), ri, 6e-2, f'gqa D{D}')


@pytest.mark.parametrize('D', [96, 256])
@pytest.mark.parametrize('causal', [False, True])
def test_wide_mask(D, causal):
    B, Sq, Sk, H = 2, 130, 200, 2
    q, k, v = _leaf(B, Sq, H, D), _leaf(B, Sk, H, D), _leaf(B, Sk, H, D)
    mask = torch.randn(B, 1, Sq, Sk, device=DEV) * 2
    mask[:, :, :, 5:40] = float('-inf')
    o = FA.flash_attention_ex(q, k, v, causal, mask=mask)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal, mask=mask)
    _close(o, r, 2e-2, name='wide mask fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'wide mask')


@pytest.mark.parametrize('D', [96, 256])
def test_wide_dropout(D):
    B, S, H, p = 1, D, 2, 0.25
    q, k, v, o, z = _dropout_mask(B, S, H, D, True, p, seed=11)
    kept = (z[..., torch.ones(S, S, device=DEV, dtype=torch.bool).tril()] > 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.04, kept
    _close(o, _ref(q, k, v, True, z=z), 2e-2, name='wide dropout fwd')
    qq, kk, vv = _leaf(B, S, H, D, scale=0.3), _leaf(B, S, H, D, scale=0.3), _leaf(B, S, H, D)
    torch.manual_seed(11)
    o2 = FA.flash_attention_ex(qq, kk, vv, True, dropout=p)
    ri = [t.detach().float().requires_grad_() for t in (qq, kk, vv)]
    r = _ref(*ri, True, z=z)
    _close(o2, r, 3e-2, name='wide dropout fwd2')
    _grads_vs_ref(o2, r, (qq, kk, vv), ri, 6e-2, 'wide dropout')


@pytest.mark.parametrize('D', [96, 256])
def test_wide_varlen(D):
    lens = [37, 128, 1, 200]
    cu = torch.tensor([0] + lens, device=DEV).cumsum(0).int()
    q, k, v = _leaf(sum(lens), 4, D), _leaf(sum(lens), 2, D), _leaf(sum(lens), 2, D)
    o = FA.flash_attention_ex(q, k, v, True, cu_seqlens_q=cu, cu_seqlens_k=cu)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = torch.cat([_ref(ri[0][a:b][None], ri[1][a:b][None], ri[2][a:b][None], True)[0]
                   for a, b in zip(cu[:-1].tolist(), cu[1:].tolist())])
    _close(o, r, 2e-2, name='wide varlen fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'wide varlen')


@pytest.mark.parametrize('D', [96, 256])
def test_wide_flashmask_rows(D):
    B, S, H = 1, 260, 2
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    rows = torch.randint(S // 3, S + 1, (B, 1, S), device=DEV, dtype=torch.int32)
    rows[..., 0] = S
    o = FA.flash_attention_ex(q, k, v, True, start_rows=rows)
    keep = torch.arange(S, device=DEV).view(1, 1, S, 1) < rows.unsqueeze(2)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, True, mask=keep)
    _close(o, r, 2e-2, name='wide flashmask fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'wide flashmask')


@pytest.mark.parametrize('D,Dk', [(96, 96), (256, 256), (80, 96), (192, 256)])
def test_api_wide_head_dims_hit_kernel(D, Dk, monkeypatch):
    """paddle.nn.functional.flash_attention with head dims 96 / 256 runs the native tile (80 and
    192 pad to them), never the S^2 composite."""
    import sys
    M = sys.modules[paddle.nn.functional.flash_attention.__module__]
    monkeypatch.setattr(M, '_sdpa_reference', lambda *a, **k: (_ for _ in ()).throw(AssertionError('composite')))
    B, S, H = 2, 160, 2
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    from paddle.core.tensor import _wrap
    out, _ = paddle.nn.functional.flash_attention(_wrap(q), _wrap(k), _wrap(v), causal=True)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, True)
    _close(out._t, r, 2e-2, name=f'api D{D}')
    _grads_vs_ref(out._t, r, (q, k, v), ri, 5e-2, f'api D{D}')
    assert FA.tiled_head_dim(D) == Dk
