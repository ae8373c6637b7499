"""GPU numerics of the software-pipelined flash-attention forward (csrc/flash_attn_kernels.h
fwd_sp_kernel: S(kb+1) on the matrix pipe while the softmax of S(kb) runs, K/V by LDS-DMA into
two-slot rings) against fp32 PyTorch and against the classic forward kernel, over causal /
non-causal, ragged lengths, GQA, additive and bool masks, dropout (same keep mask) and varlen."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402,F401
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

DEV = 'cuda'
FA = ops.flash_attn


def setup_module(m):
    assert _native._load() is not None, _native.load_error


class _SP:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.old = _native.lib.pa_flash_set_fwd_sp(int(self.on))

    def __exit__(self, *a):
        _native.lib.pa_flash_set_fwd_sp(self.old)


def _ref(q, k, v, causal, mask=None):
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if kf.shape[1] != qf.shape[1]:
        rep = qf.shape[1] // kf.shape[1]
        kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if mask is not None:
        s = s.masked_fill(~mask, float('-inf')) if mask.dtype == torch.bool else s + mask.float()
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1 + Sk - Sq), float('-inf'))
    return torch.nan_to_num(torch.softmax(s, -1), nan=0.0).matmul(vf).transpose(1, 2)


def _rand(*shape, dt=torch.bfloat16):
    return torch.randn(*shape, device=DEV).to(dt)


@pytest.mark.parametrize('causal', [False, True])
@pytest.mark.parametrize('B,Sq,Sk,H,Hk', [(2, 512, 512, 4, 4), (1, 333, 333, 2, 2), (2, 200, 517, 4, 2),
                                          (1, 64, 64, 2, 2), (3, 1024, 1024, 2, 1)])
@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
def test_sp_forward_matches_fp32_and_classic(causal, B, Sq, Sk, H, Hk, dt):
    torch.manual_seed(B * 7 + Sq)
    q, k, v = _rand(B, Sq, H, 64, dt=dt), _rand(B, Sk, Hk, 64, dt=dt), _rand(B, Sk, Hk, 64, dt=dt)
    with torch.no_grad():
        with _SP(True):
            o_sp = FA.flash_attention(q, k, v, causal)
        with _SP(False):
            o_cl = FA.flash_attention(q, k, v, causal)
    ref = _ref(q, k, v, causal)
    assert torch.isfinite(o_sp.float()).all()
    assert (o_sp.float() - ref).abs().max().item() < 2e-2
    assert (o_sp.float() - o_cl.float()).abs().max().item() < 1e-2


@pytest.mark.parametrize('kind', ['bool', 'add'])
def test_sp_forward_masks_and_dropout(kind):
    torch.manual_seed(3)
    B, S, H = 4, 512, 12
    q, k, v = (_rand(B, S, H, 64) for _ in range(3))
    keep = torch.ones(B, 1, 1, S, dtype=torch.bool, device=DEV)
    keep[1, ..., 300:] = False
    keep[3, ..., 17:] = False
    mask = keep if kind == 'bool' else torch.where(keep, 0.0, -1e4).to(torch.bfloat16)
    with torch.no_grad():
        with _SP(True):
            o = FA.flash_attention_ex(q, k, v, mask=mask)
            torch.manual_seed(11)
            od = FA.flash_attention_ex(q, k, v, mask=mask, dropout=0.1)
        with _SP(False):
            torch.manual_seed(11)
            od_cl = FA.flash_attention_ex(q, k, v, mask=mask, dropout=0.1)
    ref = _ref(q, k, v, False, keep)
    assert (o.float() - ref).abs().max().item() < 2e-2
    # dropout: the same counter-hash keep mask in both kernels
    assert (od.float() - od_cl.float()).abs().max().item() < 1e-2


def test_sp_forward_grad_through_classic_backward():
    torch.manual_seed(5)
    q, k, v = (_rand(2, 256, 4, 64).requires_grad_() for _ in range(3))
    with _SP(True):
        o = FA.flash_attention(q, k, v, True)
    g = torch.randn_like(o)
    o.backward(g)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    _ref(qr, kr, vr, True).backward(g.float())
    for a, b_, n in ((q.grad, qr.grad, 'dq'), (k.grad, kr.grad, 'dk'), (v.grad, vr.grad, 'dv')):
        assert (a.float() - b_).abs().max().item() < 5e-2, n


@pytest.mark.parametrize('sp', [0, 1])
@pytest.mark.parametrize('D', [64, 128])
def test_key_padding_mask_mixed_batch_fwd_bwd(sp, D):
    """A key-only padding mask where some batch entries are unpadded (their per-element mask loads
    are skipped through the per-batch all-keep flags) and others padded: forward and gradients vs
    fp32, through both forward kernels."""
    torch.manual_seed(21 + D)
    B, S, H = 4, 320, 4
    q, k, v = (torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16).requires_grad_() for _ in range(3))
    keep = torch.ones(B, 1, 1, S, dtype=torch.bool, device=DEV)
    keep[1, ..., 250:] = False
    keep[2, ..., 7:] = False
    with _SP(bool(sp)):
        o = FA.flash_attention_ex(q, k, v, mask=keep)
    g = torch.randn_like(o)
    o.backward(g)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, False, keep)
    ref.backward(g.float())
    assert (o.float() - ref).abs().max().item() < 2e-2
    for a, b_, n in ((q.grad, qr.grad, 'dq'), (k.grad, kr.grad, 'dk'), (v.grad, vr.grad, 'dv')):
        assert (a.float() - b_).abs().max().item() < 6e-2, n
