"""Flash-attention backward through a materialised dS (csrc/flash_attn_ds.hip: delta pass, dK/dV
kernel storing dS^T, dQ = dS K): gradients of every feature against the fp32 reference, and
against the recompute backward (flash_attn.hip) for dropout, whose keep mask only the kernels know."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402,F401
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

from test_hip_flash_ex import _close, _ref, _leaf, _grads_vs_ref  # noqa: E402

DEV = 'cuda'
FA = ops.flash_attn


def setup_module(m):
    torch.manual_seed(0)
    assert _native._load() is not None, _native.load_error


@pytest.fixture
def ds_on():
    old = FA.set_ds_backward(True)
    yield
    FA.set_ds_backward(old)


@pytest.mark.parametrize('D', [64, 128])
@pytest.mark.parametrize('causal', [False, True])
@pytest.mark.parametrize('S', [128, 200, 1024])
def test_ds_plain(ds_on, D, causal, S):
    B, H = 2, 4
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    o = FA.flash_attention(q, k, v, causal)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal)
    _close(o, r, 2e-2, name='fwd')
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, f'ds D{D}')


def test_ds_packed_gqa_cross(ds_on):
    B, S, H, D = 2, 256, 4, 128
    qkv = _leaf(B, S, 3, H, D)
    o = FA.flash_attention_packed(qkv, True)
    ri = qkv.detach().float().requires_grad_()
    r = _ref(ri[:, :, 0], ri[:, :, 1], ri[:, :, 2], True)
    g = torch.randn_like(r)
    o.backward(g.bfloat16())
    r.backward(g)
    _close(qkv.grad, ri.grad, 6e-2, 2e-2, 'packed')
    q, k, v = _leaf(2, 150, 8, 64), _leaf(2, 333, 2, 64), _leaf(2, 333, 2, 64)
    for causal in (False, True):
        for t in (q, k, v):
            t.grad = None
        o = FA.flash_attention(q, k, v, causal)
        ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
        r = _ref(*ri, causal)
        _grads_vs_ref(o, r, (q, k, v), ri, 6e-2, f'gqa cross causal={causal}')


@pytest.mark.parametrize('causal', [False, True])
def test_ds_mask_varlen_flashmask(ds_on, causal):
    B, Sq, Sk, H, D = 2, 200, 264, 4, 128
    q, k, v = _leaf(B, Sq, H, D), _leaf(B, Sk, H, D), _leaf(B, Sk, H, D)
    mask = torch.randn(B, 1, Sq, Sk, device=DEV) * 2
    mask[:, :, :, 5:40] = float('-inf')
    o = FA.flash_attention_ex(q, k, v, causal, mask=mask)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal, mask=mask)
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'ds mask')
    lens = [37, 128, 1, 200]
    cu = torch.tensor([0] + lens, device=DEV).cumsum(0).int()
    q, k, v = _leaf(sum(lens), 4, 64), _leaf(sum(lens), 2, 64), _leaf(sum(lens), 2, 64)
    o = FA.flash_attention_ex(q, k, v, causal, cu_seqlens_q=cu, cu_seqlens_k=cu)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = torch.cat([_ref(ri[0][a:b][None], ri[1][a:b][None], ri[2][a:b][None], causal)[0]
                   for a, b in zip(cu[:-1].tolist(), cu[1:].tolist())])
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'ds varlen')
    S = 300
    q, k, v = _leaf(1, S, 2, 128), _leaf(1, S, 2, 128), _leaf(1, S, 2, 128)
    rows = torch.randint(S // 3, S + 1, (1, 1, S), device=DEV, dtype=torch.int32)
    rows[..., 0] = S
    o = FA.flash_attention_ex(q, k, v, causal, start_rows=rows)
    keep = torch.arange(S, device=DEV).view(1, 1, S, 1) < rows.unsqueeze(2)
    ri = [t.detach().float().requires_grad_() for t in (q, k, v)]
    r = _ref(*ri, causal, mask=keep)
    _grads_vs_ref(o, r, (q, k, v), ri, 5e-2, 'ds flashmask')


@pytest.mark.parametrize('D', [64, 128])
def test_ds_dropout_matches_recompute(D):
    """Same seed -> same keep mask in both backward forms: their gradients agree to bf16 rounding."""
    B, S, H = 2, 512, 4
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    g = torch.randn(B, S, H, D, device=DEV).bfloat16()
    grads = []
    for on in (False, True):
        old = FA.set_ds_backward(on)
        try:
            for t in (q, k, v):
                t.grad = None
            torch.manual_seed(5)
            o = FA.flash_attention_ex(q, k, v, True, dropout=0.2)
            o.backward(g)
            grads.append([t.grad.float().clone() for t in (q, k, v)])
        finally:
            FA.set_ds_backward(old)
    for a, b, n in zip(grads[0], grads[1], 'qkv'):
        _close(b, a, 3e-2, 1e-2, f'dropout d{n} ds vs recompute')


def test_ds_llama_bench_shape_strided_qkv():
    """The llama2_13b bench key's attention: B2 S4096 H40 D128 causal, q/k/v strided views of one
    [B, S, 3H, D] projection, through the dS backward (default at D = 128) vs fp32."""
    assert FA._ds_ok(128, torch.bfloat16)
    B, S, H, D = 2, 4096, 40, 128
    qkv = _leaf(B, S, 3 * H, D)
    q, k, v = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
    o = FA.flash_attention(q, k, v, True)
    ri = qkv.detach().float().requires_grad_()
    r = _ref(ri[:, :, :H], ri[:, :, H:2 * H], ri[:, :, 2 * H:], True)
    _close(o, r, 2e-2, name='llama fwd')
    g = torch.randn_like(r)
    o.backward(g.bfloat16())
    r.backward(g)
    for i, n in enumerate('qkv'):
        sl = slice(i * H, (i + 1) * H)
        _close(qkv.grad[:, :, sl], ri.grad[:, :, sl], 5e-2, 2e-2, f'llama d{n}')
    del r, ri
    torch.cuda.empty_cache()


def test_ds_workspace_survives_growth_after_capture(ds_on):
    """A graph captured with the dS backward keeps its workspace: an eager call at a larger shape
    grows the workspace, the replay must still produce the captured shape's gradients."""
    B, S, H, D = 2, 256, 4, 128
    q, k, v = _leaf(B, S, H, D), _leaf(B, S, H, D), _leaf(B, S, H, D)
    g = torch.randn(B, S, H, D, device=DEV).bfloat16()
    FA._DS_WS.release()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up on the capture stream
        for t in (q, k, v):
            t.grad = None
        FA.flash_attention(q, k, v, True).backward(g)
    torch.cuda.current_stream().wait_stream(s)
    ref = [t.grad.clone() for t in (q, k, v)]
    graph = torch.cuda.CUDAGraph()
    for t in (q, k, v):
        t.grad = torch.zeros_like(t)
    with torch.cuda.graph(graph):
        o = FA.flash_attention(q, k, v, True)
        o.backward(g)
    # larger eager shape: grows (replaces) the workspace
    big = [_leaf(4, 2048, 8, D) for _ in range(3)]
    FA.flash_attention(*big, True).backward(torch.randn(4, 2048, 8, D, device=DEV).bfloat16())
    assert FA._DS_WS.nbytes() >= 4 * 8 * 2048 * 2048 * 2
    keep = torch.full((64 << 20,), 7.0, device=DEV)  # recycle freed memory into live tensors
    for t in (q, k, v):
        t.grad.zero_()
    graph.replay()
    torch.cuda.synchronize()
    for a, b, n in zip((q, k, v), ref, 'qkv'):
        _close(a.grad, b, 1e-2, name=f'replay d{n}')
    assert bool((keep == 7.0).all())


@pytest.mark.parametrize('causal', [False, True])
def test_ds_dq_dma_ring_bitwise(ds_on, causal):
    """The LDS-DMA ring dQ kernel runs the register-staged kernel's MFMA chain
    in the same order: bitwise-equal dQ, on a ragged cross-attention shape and under varlen-free
    GQA strides."""
    q, k, v = _leaf(2, 333, 8, 128), _leaf(2, 461, 2, 128), _leaf(2, 461, 2, 128)
    g = torch.randn(2, 333, 8, 128, device=DEV, dtype=torch.bfloat16)
    got = {}
    old = _native.lib.pa_flash_ds_set_dq_dma(0)
    try:
        for mode in (0, 2):
            _native.lib.pa_flash_ds_set_dq_dma(mode)
            for t in (q, k, v):
                t.grad = None
            FA.flash_attention(q, k, v, causal).backward(g)
            got[mode] = [t.grad.clone() for t in (q, k, v)]
    finally:
        _native.lib.pa_flash_ds_set_dq_dma(old)
    for mode in (2,):
        for a, b in zip(got[0], got[mode]):
            assert torch.equal(a, b), (mode, (a.float() - b.float()).abs().max().item())
