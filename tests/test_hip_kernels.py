"""Numerics of every hand-written HIP kernel vs a plain PyTorch fp32 reference of the same op.

All tests need an MI355X; they run with the kernel library loaded (ops.use_hip raises if the
library is missing on a GPU process).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

DEV = 'cuda'


def setup_module(m):
    torch.manual_seed(0)
    assert _native._load() is not None, _native.load_error


def _close(a, b, atol, rtol=0.0, name=''):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{name}: max err {err} > {tol}"


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(64, 2048), (33, 768), (8, 4096), (5, 300), (16, 12288)])
@pytest.mark.parametrize("wdt", ['same', 'f32'])
def test_layernorm(dt, shape, wdt):
    x = torch.randn(*shape, device=DEV, dtype=dt, requires_grad=True)
    wd = dt if wdt == 'same' else torch.float32
    w = (1 + 0.1 * torch.randn(shape[-1], device=DEV)).to(wd).requires_grad_()
    b = (0.1 * torch.randn(shape[-1], device=DEV)).to(wd).requires_grad_()
    y = ops.norm.layer_norm(x, w, b, 1e-5)
    xr, wr, br = x.detach().float().requires_grad_(), w.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, [shape[-1]], wr, br, 1e-5)
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    _close(y, yr, tol, name='ln fwd')
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _close(x.grad, xr.grad, tol * 2, 2e-2, 'ln dx')
    _close(w.grad, wr.grad, tol * 4, 2e-2, 'ln dw')
    _close(b.grad, br.grad, tol * 4, 2e-2, 'ln db')


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(64, 4096), (7, 5120), (3, 100)])
def test_rmsnorm(dt, shape):
    x = torch.randn(*shape, device=DEV, dtype=dt, requires_grad=True)
    w = (1 + 0.1 * torch.randn(shape[-1], device=DEV)).to(dt).requires_grad_()
    y = ops.norm.rms_norm(x, w, 1e-6)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    _close(y, yr, tol, name='rms fwd')
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _close(x.grad, xr.grad, tol * 2, 2e-2, 'rms dx')
    _close(w.grad, wr.grad, tol * 4, 2e-2, 'rms dw')


def test_add_layernorm_residual():
    x = torch.randn(32, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(32, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(1024, device=DEV, requires_grad=True)
    b = torch.zeros(1024, device=DEV, requires_grad=True)
    y, s = ops.norm.add_layer_norm(x, r, w, b, 1e-5)
    sr = (x.detach().float() + r.detach().float()).requires_grad_()
    yr = torch.nn.functional.layer_norm(sr, [1024], None, None, 1e-5)
    _close(s, sr, 2e-2, name='sum')
    _close(y, yr, 3e-2, name='y')
    gy, gs = torch.randn_like(yr), torch.randn_like(yr)
    torch.autograd.backward([y, s], [gy.bfloat16(), gs.bfloat16()])
    (yr * gy + sr * gs).sum().backward()
    _close(x.grad, sr.grad, 6e-2, 2e-2, 'dx')
    _close(r.grad, sr.grad, 6e-2, 2e-2, 'dr')


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("cols", [128, 1000, 2048, 4097])
def test_softmax(dt, cols):
    x = (3 * torch.randn(37, cols, device=DEV)).to(dt).requires_grad_()
    y = ops.softmax.softmax(x)
    xr = x.detach().float().requires_grad_()
    yr = torch.softmax(xr, -1)
    _close(y, yr, 1e-2 if dt != torch.float32 else 1e-5, name='sm')
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _close(x.grad, xr.grad, 2e-2 if dt != torch.float32 else 1e-5, 2e-2, 'sm dx')


def test_softmax_causal():
    S = 96
    x = torch.randn(2, 4, S, S, device=DEV, dtype=torch.bfloat16)
    y = ops.softmax.softmax_mask_upper_triangle(x)
    m = torch.ones(S, S, device=DEV, dtype=torch.bool).triu(1)
    yr = torch.softmax(x.float().masked_fill(m, float('-inf')), -1)
    _close(y, yr, 1e-2, name='causal sm')


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("vocab", [50304, 1000, 777])
def test_cross_entropy(dt, vocab):
    N = 64
    logits = (2 * torch.randn(N, vocab, device=DEV)).to(dt).requires_grad_()
    lab = torch.randint(0, vocab, (N,), device=DEV)
    lab[3] = -100
    loss = ops.xent.softmax_cross_entropy(logits, lab, -100)
    lr_ = logits.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr_, lab, ignore_index=-100, reduction='none')
    _close(loss, ref, 2e-2 if dt == torch.bfloat16 else 1e-4, name='xent')
    g = torch.rand(N, device=DEV)
    loss.backward(g)
    ref.backward(g)
    _close(logits.grad, lr_.grad, 1e-2 if dt == torch.bfloat16 else 1e-5, name='xent grad')


@pytest.mark.parametrize("approx", [False, True])
def test_gelu(approx):
    x = torch.randn(1000, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.act.gelu(x, approx, bias=b)
    xr, br = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = torch.nn.functional.gelu(xr + br, approximate='tanh' if approx else 'none')
    _close(y, yr, 3e-2, name='gelu')
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    _close(x.grad, xr.grad, 3e-2, 2e-2, 'gelu dx')
    _close(b.grad, br.grad, 1.0, 2e-2, 'gelu db')


def test_silu_swiglu():
    a = torch.randn(64, 2, 512, device=DEV, dtype=torch.bfloat16)
    buf = torch.randn(64, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    x, gt = buf[:, :512], buf[:, 512:]
    y = ops.act.swiglu(x, gt)
    br = buf.detach().float().requires_grad_()
    yr = torch.nn.functional.silu(br[:, :512]) * br[:, 512:]
    _close(y, yr, 3e-2, name='swiglu')
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    _close(buf.grad, br.grad, 5e-2, 2e-2, 'swiglu grads')
    _ = a


def test_dropout_add():
    x = torch.randn(4096, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(4096, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    p = 0.1
    y = ops.act.dropout_add(x, r, p)
    diff = y.detach().float() - r.detach().float()
    nz = x.detach().float().abs() > 0.1
    kept = (diff.abs() > 1e-6) & nz
    frac = (kept.float().sum() / nz.float().sum()).item()
    assert abs(frac - (1 - p)) < 0.01, frac
    _close(diff[kept], (x.detach().float() / (1 - p))[kept], 0.05, 0.01, 'scale')
    y.backward(torch.ones_like(y))
    # backward regenerates the identical mask from (seed, offset)
    _close(x.grad.float()[nz], (kept.float() / (1 - p))[nz], 1e-2, name='dx mask')
    _close(r.grad, torch.ones_like(r.grad), 0, name='dres')


def test_embedding():
    V, D = 50304, 2048
    w = (torch.randn(V, D, device=DEV) * 0.02).bfloat16().requires_grad_()
    ids = torch.randint(0, V, (8, 128), device=DEV)
    ids[0, :10] = 5  # repeated ids accumulate
    y = ops.embedding.embedding(ids, w)
    _close(y, w.detach()[ids], 0, name='emb fwd')
    g = torch.randn(8, 128, D, device=DEV, dtype=torch.bfloat16)
    y.backward(g)
    ref = torch.zeros(V, D, device=DEV).index_add_(0, ids.reshape(-1), g.reshape(-1, D).float())
    _close(w.grad, ref, 5e-2, 1e-2, 'emb grad')


@pytest.mark.parametrize("interleaved", [False, True])
def test_rope(interleaved):
    from paddle.incubate.nn.functional import _rope_ref
    B, S, H, D = 2, 64, 4, 128
    x = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    c, s = ops.rope.rope_tables(S, D, 10000.0, x.device)
    y = ops.rope.apply_rope(x, c, s, None, interleaved)
    xr = x.detach().float().requires_grad_()
    yr = _rope_ref(xr, c, s, None, interleaved)
    _close(y, yr, 3e-2, name='rope')
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    _close(x.grad, xr.grad, 3e-2, name='rope bwd')


def test_adamw_flat_matches_reference():
    n = 10007
    p32 = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV).bfloat16()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    low = p32.bfloat16()
    ref_p, ref_m, ref_v = p32.clone(), m.clone(), v.clone()
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.95, 1e-8, 0.1
    b1p, b2p = b1, b2
    for _ in range(3):
        ops.optim.adamw_flat(p32, g, m, v, low, lr, b1, b2, eps, wd, b1p, b2p)
        gg = g.float()
        ref_p.mul_(1 - lr * wd)
        ref_m.mul_(b1).add_((1 - b1) * gg)
        ref_v.mul_(b2).add_((1 - b2) * gg * gg)
        ref_p.sub_(lr * math.sqrt(1 - b2p) / (1 - b1p) * ref_m / (ref_v.sqrt() + eps * math.sqrt(1 - b2p)))
        b1p *= b1
        b2p *= b2
    _close(p32, ref_p, 1e-6, name='adamw p')
    _close(m, ref_m, 1e-6, name='adamw m')
    _close(low, ref_p, 2e-2, name='adamw lowp')


def _attn_ref(q, k, v, causal):
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if kf.shape[1] != qf.shape[1]:
        rep = qf.shape[1] // kf.shape[1]
        kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        Sq, Sk = s.shape[-2:]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1 + Sk - Sq)
        s = s.masked_fill(m, float('-inf'))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("S", [128, 200, 1024])
def test_flash_attention_fwd_bwd(D, causal, S):
    B, H = 2, 4
    q = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attn.flash_attention(q, k, v, causal)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _attn_ref(qr, kr, vr, causal)
    _close(o, orf, 2e-2, name='fa fwd')
    g = torch.randn_like(orf)
    o.backward(g.bfloat16())
    orf.backward(g)
    _close(q.grad, qr.grad, 5e-2, 2e-2, 'dq')
    _close(k.grad, kr.grad, 5e-2, 2e-2, 'dk')
    _close(v.grad, vr.grad, 5e-2, 2e-2, 'dv')


def test_flash_attention_strided_qkv_gqa():
    B, S, H, Hk, D = 2, 256, 8, 2, 128
    qkv = torch.randn(B, S, H + 2 * Hk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    q, k, v = qkv[:, :, :H], qkv[:, :, H:H + Hk], qkv[:, :, H + Hk:]
    o = ops.flash_attn.flash_attention(q, k, v, True)
    ref_in = qkv.detach().float().requires_grad_()
    orf = _attn_ref(ref_in[:, :, :H], ref_in[:, :, H:H + Hk], ref_in[:, :, H + Hk:], True)
    _close(o, orf, 2e-2, name='gqa fwd')
    g = torch.randn_like(orf)
    o.backward(g.bfloat16())
    orf.backward(g)
    _close(qkv.grad, ref_in.grad, 6e-2, 2e-2, 'gqa grads')


def test_flash_attention_packed_qkv():
    B, S, H, D = 2, 512, 4, 128
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attn.flash_attention_packed(qkv, True)
    ref_in = qkv.detach().float().requires_grad_()
    orf = _attn_ref(ref_in[:, :, 0], ref_in[:, :, 1], ref_in[:, :, 2], True)
    _close(o, orf, 2e-2, name='packed fwd')
    g = torch.randn_like(orf)
    o.backward(g.bfloat16())
    orf.backward(g)
    _close(qkv.grad, ref_in.grad, 6e-2, 2e-2, 'packed grads')


def test_flash_attention_cross_lengths():
    B, H, D = 1, 2, 64
    q = torch.randn(B, 100, H, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, 300, H, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, 300, H, D, device=DEV, dtype=torch.bfloat16)
    for causal in (False, True):
        o = ops.flash_attn.flash_attention(q, k, v, causal)
        _close(o, _attn_ref(q, k, v, causal), 2e-2, name=f'cross causal={causal}')


def test_paddle_api_routes_to_hip():
    x = paddle.randn([4, 256, 8, 64]).astype('bfloat16')
    out, _ = paddle.nn.functional.flash_attention(x, x, x, causal=True)
    ref = _attn_ref(x._t, x._t, x._t, True)
    _close(out._t, ref, 2e-2, name='api fa')
    h = paddle.randn([16, 1024]).astype('bfloat16')
    ln = paddle.nn.LayerNorm(1024)
    ln.to(dtype='bfloat16')
    _close(ln(h)._t, torch.nn.functional.layer_norm(h._t.float(), [1024]), 3e-2, name='api ln')


def test_gpt_tiny_train_step_gpu():
    from paddle.models.gpt import gpt_config, GPTForPretraining
    paddle.seed(0)
    cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0)
    model = GPTForPretraining(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters(), multi_precision=True)
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    ids = paddle.randint(0, cfg.vocab_size, [4, 65])
    x, y = ids[:, :-1], ids[:, 1:]
    losses = []
    for _ in range(20):
        loss = model.loss(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,off", [(1, 0), (37, 3), (100003, 5), (1 << 22, 0)])
def test_sumsq_vectorized(dt, n, off):
    buf = torch.randn(n + off, device=DEV, dtype=dt)
    x = buf[off:]
    got = ops.optim.sumsq(x)
    ref = x.float().pow(2).sum()
    assert abs(float(got) - float(ref)) <= 1e-4 * float(ref) + 1e-5
