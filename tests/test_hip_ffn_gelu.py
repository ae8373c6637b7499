"""Fused feed-forward autograd op of static training programs (ops.matmul.ffn_gelu, the
fuse_gemm_epilogue_pass target): fc1's GEMM epilogue writes gelu(h) and gelu'(h) (exact erf form:
csrc/gemm8.hip epi 9; tanh form: epi 2), the fc2 data-gradient GEMM multiplies by gelu'(h) and
reduces the fc1 bias gradient in its epilogue — values and all five gradients vs fp32 torch."""
import pytest
import torch

import paddle  # noqa: F401
from paddle.ops import matmul as HM

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('approximate', [False, True])
@pytest.mark.parametrize('M,H,F', [(2048, 256, 1024), (136, 128, 512), (4096, 768, 3072)])
def test_ffn_gelu_matches_fp32(approximate, M, H, F):
    torch.manual_seed(0)
    dev = 'cuda'
    x = torch.randn(M, H, device=dev).bfloat16().requires_grad_()
    w1 = (torch.randn(H, F, device=dev) * H ** -0.5).bfloat16().requires_grad_()
    b1 = (torch.randn(F, device=dev) * 0.5).bfloat16().requires_grad_()
    w2 = (torch.randn(F, H, device=dev) * F ** -0.5).bfloat16().requires_grad_()
    b2 = (torch.randn(H, device=dev) * 0.5).bfloat16().requires_grad_()
    assert HM.ffn_gelu_ok(x, w1, b1, w2, b2)
    y = HM.ffn_gelu(x, w1, b1, w2, b2, approximate)
    dy = torch.randn(M, H, device=dev).bfloat16()
    y.backward(dy)
    ref_in = [t.detach().float().requires_grad_() for t in (x, w1, b1, w2, b2)]
    xr, w1r, b1r, w2r, b2r = ref_in
    yr = torch.nn.functional.gelu(xr @ w1r + b1r, approximate='tanh' if approximate else 'none') @ w2r + b2r
    yr.backward(dy.float())

    def rel(a, b):
        return ((a.float() - b).norm() / b.norm()).item()
    assert rel(y, yr) < 1e-2, rel(y, yr)
    for name, t, r in zip(('dx', 'dw1', 'db1', 'dw2', 'db2'), (x, w1, b1, w2, b2), ref_in):
        e = rel(t.grad, r.grad)
        assert e < 2e-2, (name, e)


def test_ffn_gelu_contract_rejects():
    dev = 'cuda'
    x = torch.randn(100, 64, device=dev).bfloat16()  # rows % 8 != 0
    w1, b1 = torch.randn(64, 256, device=dev).bfloat16(), torch.randn(256, device=dev).bfloat16()
    w2, b2 = torch.randn(256, 64, device=dev).bfloat16(), torch.randn(64, device=dev).bfloat16()
    assert not HM.ffn_gelu_ok(x, w1, b1, w2, b2)
    assert not HM.ffn_gelu_ok(x[:96].float(), w1, b1, w2, b2)
    assert HM.ffn_gelu_ok(x[:96].contiguous(), w1, b1, w2, b2)


@pytest.mark.parametrize('approximate', [False, True])
def test_fp8_ffn_matches_unfused_fp8_linears(approximate):
    """ops.fp8.fp8_ffn (fp8 GEMMs with the GELU / GELU' epilogues) vs two fp8 Linears around a
    torch GELU, both under delayed scaling from fresh states, and vs fp32."""
    from paddle.ops import fp8 as F8
    torch.manual_seed(3)
    M, H, F = 2048, 256, 1024
    dev = 'cuda'

    def leaf(t):
        return t.bfloat16().requires_grad_()
    x = leaf(torch.randn(M, H, device=dev))
    w1, b1 = leaf(torch.randn(H, F, device=dev) * H ** -0.5), leaf(torch.randn(F, device=dev) * 0.5)
    w2, b2 = leaf(torch.randn(F, H, device=dev) * F ** -0.5), leaf(torch.randn(H, device=dev) * 0.5)
    ps = (x, w1, b1, w2, b2)
    assert F8.ffn_ok(*ps)
    dy = torch.randn(M, H, device=dev).bfloat16()
    rec = F8.DelayedScaling(amax_history_len=4)
    F8._STATIC_STATES.clear()
    y = F8.fp8_ffn(*ps, approximate=approximate, recipe=rec)
    y.backward(dy)
    g_fused = [p.grad.float().clone() for p in ps]
    for p in ps:
        p.grad = None
    F8._STATIC_STATES.clear()
    act = 'tanh' if approximate else 'none'
    h = F8.fp8_linear(x, w1, b1, recipe=rec)
    yu = F8.fp8_linear(torch.nn.functional.gelu(h, approximate=act), w2, b2, recipe=rec)
    yu.backward(dy)
    g_unf = [p.grad.float() for p in ps]
    ref = [p.detach().float().requires_grad_() for p in ps]
    yr = torch.nn.functional.gelu(ref[0] @ ref[1] + ref[2], approximate=act) @ ref[3] + ref[4]
    yr.backward(dy.float())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()
    assert rel(y, yu) < 3e-2 and rel(y, yr) < 8e-2, (rel(y, yu), rel(y, yr))
    for name, gf, gu, r in zip(('dx', 'dw1', 'db1', 'dw2', 'db2'), g_fused, g_unf, ref):
        assert rel(gf, gu) < 6e-2 and rel(gf, r.grad) < 1.2e-1, (name, rel(gf, gu), rel(gf, r.grad))


def test_fp8_ffn_fused_quantisation_matches_cast_path(monkeypatch):
    """Once the amax histories are seeded, the fp8 FFN quantises gelu(h) (fc1 epilogue, e4m3) and
    dh (fc2 data-gradient epilogue, e5m2) inside the GEMMs (pa_gemm8_fp8_epi_q, no cast kernel);
    three steps fused vs the bf16-output + cast path from the same fresh states."""
    from paddle.ops import fp8 as F8
    torch.manual_seed(4)
    M, H, F = 2048, 256, 1024
    dev = 'cuda'
    base = [torch.randn(M, H, device=dev), torch.randn(H, F, device=dev) * H ** -0.5,
            torch.randn(F, device=dev) * 0.5, torch.randn(F, H, device=dev) * F ** -0.5,
            torch.randn(H, device=dev) * 0.5]
    dy = torch.randn(M, H, device=dev).bfloat16()
    calls = []
    orig = F8._fp8_epi_q

    def spy(*a, **k):
        r = orig(*a, **k)
        calls.append(r is not None)
        return r
    monkeypatch.setattr(F8, '_fp8_epi_q', spy)

    def run(fused):
        monkeypatch.setattr(F8, 'FUSED_QUANT', fused)
        F8._STATIC_STATES.clear()
        rec = F8.DelayedScaling(amax_history_len=4)
        ps = [t.bfloat16().requires_grad_() for t in base]
        for _ in range(3):
            for p in ps:
                p.grad = None
            y = F8.fp8_ffn(*ps, approximate=False, recipe=rec)
            y.backward(dy)
        return y.detach().float(), [p.grad.float() for p in ps]
    yf, gf = run(True)
    assert any(calls), "fused quantisation never ran"
    yu, gu = run(False)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()
    assert rel(yf, yu) < 3e-2, rel(yf, yu)
    for name, a, b in zip(('dx', 'dw1', 'db1', 'dw2', 'db2'), gf, gu):
        assert rel(a, b) < 6e-2, (name, rel(a, b))


@pytest.mark.parametrize('M,N', [(768, 3072), (768, 768)])
def test_fp8_uneven_splitk_weight_gradient(M, N):
    """fp8 weight-gradient GEMM over 32768 tokens with an uneven split-K (ops/gemm.py _fp8_splitk:
    7 / 26 slices, the last one shorter), beta = 1 accumulation, vs the fp32 product of the
    dequantised operands."""
    from paddle.ops import gemm as G, fp8 as F8
    torch.manual_seed(5)
    K = 32768
    s = G._fp8_splitk(M, N, K)
    assert s > 1 and (K // 128) % s != 0, s
    a = (torch.randn(M, K, device='cuda') * 0.5).to(F8.E4M3)
    b = (torch.randn(N, K, device='cuda') * 0.5).to(F8.E5M2)
    one = torch.ones(1, device='cuda')
    out = torch.randn(M, N, device='cuda').bfloat16()
    ref = out.float() + a.float() @ b.float().t()
    G.hip_fp8_mm(a, b, scale_a=one, scale_b=one, out=out, beta=1.0)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
