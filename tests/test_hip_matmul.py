"""The hand-written GEMM as the default dense matmul (ops/matmul.py, csrc/gemm8x.hip): batched /
broadcast / transposed bf16 and fp16 matmuls, einsum contractions, F.linear outside the training
engines (no_grad and autograd), addmm, static-graph replay, and the 8-phase fp8 GEMM — each against
a plain PyTorch fp32 reference of the same op.  Every test also asserts that the HIP kernel ran
(no library fallback) by counting pa_gemmx / skinny / hip_mm launches."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
from paddle.ops import _native, matmul as hm, gemm  # noqa: E402

DEV = 'cuda'


def setup_module(m):
    assert _native._load() is not None, _native.load_error


def _close(a, b, tol, name=''):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale, f"{name}: max err {err} > {tol} * {scale}"


class _Count:
    """Counts launches of the hand-written GEMM entry points while active."""

    def __init__(self):
        self.n = 0

    def __enter__(self):
        self._gx, self._mm, self._sk = hm._gemmx, gemm.hip_mm, gemm.skinny_mm

        def gx(*a, **k):
            r = self._gx(*a, **k)
            self.n += r is not None
            return r

        def mm(*a, **k):
            self.n += 1
            return self._mm(*a, **k)

        def sk(*a, **k):
            self.n += 1
            return self._sk(*a, **k)
        hm._gemmx, gemm.hip_mm, gemm.skinny_mm = gx, mm, sk
        return self

    def __exit__(self, *exc):
        hm._gemmx, gemm.hip_mm, gemm.skinny_mm = self._gx, self._mm, self._sk


def _rand(*shape, dt=torch.bfloat16, g=None):
    return (torch.rand(*shape, device=DEV, generator=g) * 2 - 1).to(dt)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('case', [
    ('2d', (512, 256), (256, 384)),
    ('nd_x_2d', (4, 128, 256), (256, 512)),
    ('batched', (6, 256, 128), (6, 128, 320)),
    ('bcast_b', (3, 4, 256, 64), (1, 4, 64, 256)),
    ('bcast_a', (256, 128), (5, 128, 192)),
    ('attn_qk', (2, 8, 256, 64), (2, 8, 64, 256)),
])
@pytest.mark.parametrize('tx', [False, True])
@pytest.mark.parametrize('ty', [False, True])
def test_matmul_layouts(dt, case, tx, ty):
    g = torch.Generator(device=DEV).manual_seed(1)
    _, sa, sb = case
    a = _rand(*sa, dt=dt, g=g)
    b = _rand(*sb, dt=dt, g=g)
    if tx:  # the same logical operand, stored transposed
        a = a.transpose(-1, -2).contiguous().transpose(-1, -2)
    if ty:
        b = b.transpose(-1, -2).contiguous().transpose(-1, -2)
    ref = torch.matmul(a.float(), b.float())
    with _Count() as c:
        out = hm.matmul(a, b)
    assert c.n >= 1, 'hand-written GEMM did not run'
    assert out.dtype == dt and out.shape == ref.shape
    _close(out, ref, 1e-2, f'{case[0]} {dt} tx={tx} ty={ty}')


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
def test_paddle_matmul_api_and_grad(dt):
    """paddle.matmul (transpose flags) / bmm / @ with autograd: forward and both gradients of
    broadcast batched operands vs fp32 torch autograd."""
    g = torch.Generator(device=DEV).manual_seed(2)
    a0 = _rand(3, 2, 128, 192, dt=dt, g=g)
    b0 = _rand(2, 256, 192, dt=dt, g=g)  # used transposed, broadcast over the leading 3
    a = paddle.to_tensor(a0, stop_gradient=False)
    b = paddle.to_tensor(b0, stop_gradient=False)
    with _Count() as c:
        y = paddle.matmul(a, b, transpose_y=True)
        (y.astype('float32') ** 2).sum().backward()
    assert c.n >= 3
    af = a0.float().requires_grad_()
    bf = b0.float().requires_grad_()
    yr = torch.matmul(af, bf.transpose(-1, -2))
    (yr ** 2).sum().backward()
    _close(y._t, yr, 1e-2, 'fwd')
    _close(a.grad._t, af.grad, 2e-2, 'da')
    _close(b.grad._t, bf.grad, 2e-2, 'db (reduced over the broadcast dim)')
    x = paddle.to_tensor(_rand(8, 64, 128, dt=dt, g=g))
    w = paddle.to_tensor(_rand(8, 128, 64, dt=dt, g=g))
    _close(paddle.bmm(x, w)._t, torch.bmm(x._t.float(), w._t.float()), 1e-2, 'bmm')
    _close((x @ w)._t, torch.bmm(x._t.float(), w._t.float()), 1e-2, '@')


@pytest.mark.parametrize('eq,sx,sy', [
    ('bij,jk->bik', (4, 128, 256), (256, 64)),
    ('bhqd,bhkd->bhqk', (2, 4, 128, 64), (2, 4, 128, 64)),
    ('bhqk,bhkd->bhqd', (2, 4, 128, 128), (2, 4, 128, 64)),
    ('ij,kj->ik', (256, 128), (192, 128)),
    ('bsh,hd->bsd', (2, 64, 128), (128, 256)),
])
def test_einsum_contractions(eq, sx, sy):
    g = torch.Generator(device=DEV).manual_seed(3)
    x, y = _rand(*sx, g=g), _rand(*sy, g=g)
    with _Count() as c:
        out = paddle.einsum(eq, paddle.to_tensor(x), paddle.to_tensor(y))._t
    assert c.n >= 1
    _close(out, torch.einsum(eq, x.float(), y.float()), 1e-2, eq)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
def test_linear_eval_and_train_outside_engines(dt):
    """nn.Linear without the training engines: no_grad (eval / inference) and autograd both run
    the three GEMMs on the hand-written kernel; bias fused in the epilogue."""
    paddle.seed(4)
    lin = paddle.nn.Linear(256, 512)
    lin.to(dtype='bfloat16' if dt == torch.bfloat16 else 'float16')
    x0 = _rand(4, 96, 256, dt=dt, g=torch.Generator(device=DEV).manual_seed(5))
    w, b = lin.weight._t, lin.bias._t
    ref = (x0.float() @ w.float() + b.float()).detach()
    with paddle.no_grad(), _Count() as c:
        y = lin(paddle.to_tensor(x0))
    assert c.n == 1
    _close(y._t, ref, 1e-2, 'no_grad linear')
    x = paddle.to_tensor(x0, stop_gradient=False)
    with _Count() as c:
        y = lin(x)
        y.astype('float32').sum().backward()
    assert c.n >= 3
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x0, w, b))
    (xf @ wf + bf).sum().backward()
    _close(x.grad._t, xf.grad, 2e-2, 'dx')
    _close(lin.weight.grad._t, wf.grad, 2e-2, 'dW')
    _close(lin.bias.grad._t, bf.grad, 2e-2, 'db')


def test_addmm_and_skinny_decode_shape():
    g = torch.Generator(device=DEV).manual_seed(6)
    inp = _rand(512, g=g)
    x, y = _rand(64, 1024, g=g), _rand(1024, 512, g=g)
    with torch.no_grad(), _Count() as c:
        out = paddle.addmm(paddle.to_tensor(inp), paddle.to_tensor(x), paddle.to_tensor(y))._t
    assert c.n == 1
    _close(out, inp.float() + x.float() @ y.float(), 1e-2, 'addmm')
    full = _rand(256, 512, g=g)
    x2 = _rand(256, 1024, g=g)
    with torch.no_grad(), _Count() as c:
        out = paddle.addmm(paddle.to_tensor(full), paddle.to_tensor(x2), paddle.to_tensor(y), beta=0.5, alpha=2.0)._t
    assert c.n == 1
    _close(out, 0.5 * full.float() + 2.0 * (x2.float() @ y.float()), 1e-2, 'addmm beta/alpha')


def test_addmm_leaves_input_unchanged():
    """addmm with a contiguous [M, N] input must not write its result into the input's storage."""
    g = torch.Generator(device=DEV).manual_seed(16)
    inp = _rand(256, 512, g=g)
    keep = inp.clone()
    x, y = _rand(256, 1024, g=g), _rand(1024, 512, g=g)
    with torch.no_grad():
        out = hm.addmm(inp, x, y, beta=0.5, alpha=2.0)
    assert torch.equal(inp, keep), 'addmm overwrote its input'
    assert out.data_ptr() != inp.data_ptr()
    _close(out, 0.5 * keep.float() + 2.0 * (x.float() @ y.float()), 1e-2, 'addmm fresh out')


def test_weight_only_linear_grad_reaches_x():
    """Decode-shaped weight_only_linear with x requiring grad takes the differentiable path."""
    from paddle.nn.quant import weight_quantize, weight_only_linear
    from paddle.nn.quant.quantized_linear import _dequant
    g = torch.Generator(device=DEV).manual_seed(17)
    w = torch.randn(512, 256, device=DEV, generator=g) * 0.05
    q, s = weight_quantize(paddle.to_tensor(w), algo='weight_only_int8')
    x = paddle.to_tensor(torch.randn(4, 512, device=DEV, generator=g).bfloat16())
    x.stop_gradient = False
    y = weight_only_linear(x, q, weight_scale=s, weight_dtype='int8')
    y.sum().backward()
    wd = _dequant(q, s, 'weight_only_int8', -1)
    _close(x.grad._t, wd.sum(1).expand(4, -1), 3e-2, 'woq dx')


def test_static_executor_replays_on_hip_gemm(static_mode):
    """A static Program with fc layers run by the Executor on the GPU: the recorded torch GEMM nodes
    replay on the hand-written kernel."""
    import numpy as np
    paddle.set_device('gpu:0')
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data('x', [None, 256], 'float32')
        h = paddle.static.nn.fc(x, 512)
        y = paddle.matmul(h.astype('bfloat16'), paddle.ones([512, 128], 'bfloat16'))
    exe = paddle.static.Executor(paddle.CUDAPlace(0))
    exe.run(start)
    xn = np.random.rand(64, 256).astype('float32')
    with _Count() as c:
        out, hv = exe.run(main, feed={'x': xn}, fetch_list=[y, h])
    assert c.n >= 1, 'recorded bf16 matmul did not replay on the hand-written GEMM'
    ref = torch.from_numpy(hv).bfloat16().float() @ torch.ones(512, 128)
    _close(torch.from_numpy(np.asarray(out, dtype=np.float32)), ref, 1e-2, 'static replay')


@pytest.mark.parametrize('M,N,K', [(4096, 6144, 2048), (4096, 2048, 8192), (1000, 1024, 512), (256, 4096, 1024),
                                   (768, 2304, 8192), (512, 768, 4096)])
@pytest.mark.parametrize('fmts', [(torch.float8_e4m3fn, torch.float8_e4m3fn), (torch.float8_e5m2, torch.float8_e4m3fn)])
def test_fp8_8phase_gemm(M, N, K, fmts):
    """(768 x 2304 x 8192 and 512 x 768 x 4096: the split-K path of the fp8 weight gradient)"""
    """The 8-phase fp8 GEMM (one scaled MFMA per 128-byte k-tile, device scales, bias, beta) vs the
    fp32 product of the dequantised operands."""
    g = torch.Generator(device=DEV).manual_seed(7)
    a = (torch.randn(M, K, device=DEV, generator=g) * 2).to(fmts[0])
    w = (torch.randn(N, K, device=DEV, generator=g) * 2).to(fmts[1])
    sa = torch.tensor([0.5], device=DEV)
    sb = torch.tensor([0.25], device=DEV)
    bias = _rand(N, g=g)
    assert _native.lib.pa_gemm8_fp8_ok(M, N, K, K, K, N)
    out = gemm.hip_fp8_mm(a, w, scale_a=sa, scale_b=sb, bias=bias)
    ref = (a.float() @ w.float().t()) * 0.125 + bias.float()
    _close(out, ref, 1e-2, f'fp8 {M}x{N}x{K}')
    # accumulate: out2 = 0.5 * a @ w^T * scales + 1.0 * out
    out2 = gemm.hip_fp8_mm(a, w, scale_a=sa, scale_b=sb, out=out.clone(), alpha=0.5, beta=1.0)
    _close(out2, ref + (a.float() @ w.float().t()) * 0.0625, 1.5e-2, 'fp8 beta=1')


@pytest.mark.parametrize('bits,group', [(8, -1), (8, 64), (8, 128), (4, -1), (4, 64), (4, 128)])
@pytest.mark.parametrize('M', [1, 7, 16, 32])
@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('ct', [0, 8, 4, 2])
def test_weight_only_linear_kernel(bits, group, M, dt, ct):
    """weight_only_linear on the W8A16 / W4A16 decode kernel (csrc/woq_gemm.hip) vs the fp32 product
    with the dequantised weight (Llama-2-13B-like widths scaled down); both column-tile widths."""
    from paddle.ops import _native
    old_ct = _native.lib.pa_woq_set_ct(ct)
    try:
        _woq_case(bits, group, M, dt)
    finally:
        _native.lib.pa_woq_set_ct(old_ct)


def _woq_case(bits, group, M, dt):
    from paddle.nn.quant import weight_quantize, weight_only_linear
    g = torch.Generator(device=DEV).manual_seed(11)
    K, N_ = 2560, 1152
    w = (torch.randn(K, N_, device=DEV, generator=g) * 0.05)
    x = torch.randn(M, K, device=DEV, generator=g).to(dt)
    b = torch.randn(N_, device=DEV, generator=g).to(dt)
    algo = 'weight_only_int4' if bits == 4 else 'weight_only_int8'
    q, s = weight_quantize(paddle.to_tensor(w), algo=algo, group_size=group)
    from paddle.nn.quant.quantized_linear import _dequant
    wd = _dequant(q, s, algo, group)  # [K, N] fp32
    ref = x.float() @ wd + b.float()
    from paddle.ops import woq
    calls = []
    orig = woq.woq_linear
    woq.woq_linear = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        y = weight_only_linear(paddle.to_tensor(x), q, paddle.to_tensor(b), s,
                               weight_dtype='int4' if bits == 4 else 'int8', group_size=group)._t
    finally:
        woq.woq_linear = orig
    assert calls, 'weight-only kernel did not run'
    _close(y, ref, 2e-2, f'woq bits={bits} group={group} M={M}')


@pytest.mark.parametrize('M,N,K', [(512, 768, 1024), (1000, 4096, 2048), (8, 256, 128), (4096, 2048, 4096)])
def test_int8_mfma_gemm(M, N, K):
    """pa_gemm8_i8 (v_mfma_i32_16x16x64_i8): exact int32 sums, per-row x per-column dequant, bias,
    beta accumulate — vs the fp32 product of the int8 values."""
    from paddle.ops import int8 as I8
    g = torch.Generator(device=DEV).manual_seed(21)
    a = torch.randint(-127, 128, (M, K), device=DEV, generator=g, dtype=torch.int32).to(torch.int8)
    w = torch.randint(-127, 128, (N, K), device=DEV, generator=g, dtype=torch.int32).to(torch.int8)
    rs = torch.rand(M, device=DEV, generator=g) * 0.01
    cs = torch.rand(N, device=DEV, generator=g) * 0.01
    bias = _rand(N, g=g)
    assert I8.i8_mm_ok(a, w)
    out = I8.i8_mm(a, w, rs, cs, bias=bias)
    exact = (a.double() @ w.double().t())
    ref = (exact * rs.double()[:, None] * cs.double()[None, :]).float() + bias.float()
    _close(out, ref, 1e-2, f'int8 {M}x{N}x{K}')
    out2 = I8.i8_mm(a, w, rs, cs, out=out.clone(), beta=1.0)
    _close(out2, ref + (exact * rs.double()[:, None] * cs.double()[None, :]).float(), 1.5e-2, 'int8 beta')


@pytest.mark.parametrize('M', [1, 7, 100, 512])
@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
def test_llm_int8_linear_gpu(M, dt):
    """llm_int8_linear on the int8 MFMA GEMM + the 16-bit outlier GEMM (no host sync) vs the fp32
    LLM.int8 formula; outlier columns planted."""
    from paddle.nn.quant import weight_quantize, llm_int8_linear
    from paddle.ops import int8 as I8
    g = torch.Generator(device=DEV).manual_seed(22)
    K, N_ = 1024, 768
    w = torch.randn(K, N_, device=DEV, generator=g) * 0.05
    q, s = weight_quantize(paddle.to_tensor(w), algo='llm.int8')
    x = torch.randn(M, K, device=DEV, generator=g)
    x[:, [5, 77, 900]] *= 30.0
    x = x.to(dt)
    b = torch.randn(N_, device=DEV, generator=g).to(dt)
    calls = []
    orig = I8.i8_mm
    I8.i8_mm = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        y = llm_int8_linear(paddle.to_tensor(x), q, paddle.to_tensor(b), s, threshold=6.0)._t
    finally:
        I8.i8_mm = orig
    assert calls, 'int8 kernel did not run'
    a = x.float()
    outl = (a.abs() > 6.0).any(0)
    a_in = a.masked_fill(outl[None, :], 0.0)
    sx = a_in.abs().amax(1, keepdim=True).clamp_min(1e-12) / 127.0
    qa = torch.round(a_in / sx).clamp(-127, 127)
    qw, ws = q._t.float(), s._t.float()
    ref = (qa @ qw.t()) * sx * ws[None, :] + (a * outl.float()) @ (qw * ws[:, None]).t() + b.float()
    _close(y, ref, 3e-2, f'llm.int8 M={M} {dt}')


@pytest.mark.parametrize('M,K,n', [(32, 768, 2), (96, 1024, 3), (64, 256, 7)])
def test_tiny_n_head_on_transposed_skinny(M, K, n):
    """[M, K] @ [K, n < 8] (+ bias): the classifier-head GEMM runs as its transpose on the skinny
    kernel (csrc/skinny_gemm.hip) instead of the library."""
    g = torch.Generator(device=DEV).manual_seed(40 + n)
    x, w, b = _rand(M, K, g=g), _rand(K, n, g=g), _rand(n, g=g)
    calls = []
    orig = gemm.skinny_mm

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    gemm.skinny_mm = spy
    try:
        with torch.no_grad():
            y = hm.linear(x, w, b)
    finally:
        gemm.skinny_mm = orig
    assert calls, 'tiny-N GEMM did not reach the skinny kernel'
    assert y.shape == (M, n)
    _close(y, x.float() @ w.float() + b.float(), 2e-2, 'tiny-n')


@pytest.mark.parametrize('M,K,N,kmaj,beta,bias', [(16384, 2048, 6144, True, 0.0, False), (1000, 512, 776, True, 0.0, True),
                                                (4096, 1024, 2048, True, 1.0, False), (2048, 4096, 1024, False, 1.0, False),
                                                (520, 256, 264, False, 0.0, False)])
def test_persistent_schedule_staged_epilogue_matches(M, K, N, kmaj, beta, bias):
    """Schedule 12 (persistent, the quarter-tile wave-staged epilogue in the spare LDS) equals the
    default schedules bit for bit (same per-tile accumulation order), incl. ragged edges, bias and
    the beta = 1 weight-gradient accumulate."""
    g = torch.Generator(device=DEV).manual_seed(M + N)
    a = _rand(M, K, g=g) if kmaj else _rand(K, M, g=g).t()
    b = _rand(N, K, g=g).t()
    bb = _rand(N, g=g) if bias else None
    init = _rand(M, N, g=g)
    outs = []
    for v in (0, 12):
        old = _native.lib.pa_gemm_set_variant(v)
        try:
            out = init.clone()
            gemm.hip_mm(a, b, out=out, bias=bb, beta=beta)
            torch.cuda.synchronize()
        finally:
            _native.lib.pa_gemm_set_variant(old)
        outs.append(out)
    ref = a.float() @ b.float() + (beta * init.float()) + (bb.float() if bias else 0.0)
    _close(outs[1], ref, 2e-2, 'sched12')
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize('act', ['relu', 'gelu', 'gelu_tanh'])
@pytest.mark.parametrize('M,K,N,trans', [(1024, 768, 3072, False), (1304, 512, 768, True), (2048, 1024, 640, False)])
def test_gemm_act_epilogue(act, M, K, N, trans):
    """Inference fc epilogue (pa_gemm8_bf16_act): act(x @ W + b) in the GEMM's staged epilogue vs fp32."""
    from paddle.ops import gemm as G
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device='cuda').bfloat16()
    w = (torch.randn(N, K, device='cuda') * 0.05).bfloat16() if trans else (torch.randn(K, N, device='cuda') * 0.05).bfloat16()
    W = w.t() if trans else w
    b = torch.randn(N, device='cuda').bfloat16()
    assert G.epi_ok(x, W, N)
    y = G.mm_act(x, W, b, act)
    h = x.float() @ W.float() + b.float()
    ref = {'relu': torch.relu(h), 'gelu': torch.nn.functional.gelu(h),
           'gelu_tanh': torch.nn.functional.gelu(h, approximate='tanh')}[act]
    err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


def test_gemm_autotune_cache_picks_faster_and_matches(monkeypatch):
    """Per-shape GEMM autotune (ops/matmul.py _tuned): a plain matmul is measured once on the
    hand-written kernel and the library, the choice is cached, and either choice matches fp32."""
    from paddle.ops import matmul as HM
    monkeypatch.setitem(HM._TUNE, 'on', True)
    monkeypatch.setitem(HM._TUNE, 'cache', {})
    torch.manual_seed(0)
    a = torch.randn(2048, 1024, device='cuda').bfloat16()
    b = torch.randn(1024, 3072, device='cuda').bfloat16()
    y = HM.matmul(a, b)
    y2 = HM.matmul(a, b)
    ch = HM.tuned_choices()
    assert len(ch) == 1 and list(ch.values())[0] in ('hip', 'lib'), ch
    ref = a.float() @ b.float()
    for t in (y, y2):
        err = ((t.float() - ref).norm() / ref.norm()).item()
        assert err < 1e-2, err
    q, k = torch.randn(4, 8, 256, 64, device='cuda').bfloat16(), torch.randn(4, 8, 256, 64, device='cuda').bfloat16()
    s = HM.matmul(q, k.transpose(-1, -2))
    assert any(key[0] == 'bmm' for key in HM.tuned_choices())
    rs = q.float() @ k.float().transpose(-1, -2)
    assert ((s.float() - rs).norm() / rs.norm()).item() < 1e-2


@pytest.mark.parametrize('M,N,K,s', [(768, 3072, 32768, 7), (768, 2304, 32768, 9), (256, 512, 4160, 3)])
def test_uneven_splitk_weight_gradient(M, N, K, s):
    """Split-K with a shorter last slice (ceil(K/64/s) k-blocks per slice): the weight-gradient
    layout (both operands m/n-major, x^T @ dy) with beta = 1 accumulation, vs fp32."""
    from paddle.ops import gemm as G
    torch.manual_seed(0)
    x = torch.randn(K, M, device='cuda').bfloat16()
    dy = torch.randn(K, N, device='cuda').bfloat16()
    assert G.hip_mm_ok(x.t(), dy, s)
    out = torch.randn(M, N, device='cuda').bfloat16()
    ref = out.float() + x.float().t() @ dy.float()
    G.hip_mm(x.t(), dy, out=out, beta=1.0, splitk=s)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
