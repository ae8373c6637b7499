"""Convolution everywhere: depthwise kernels (csrc/dwconv.hip), the few-channel stem forward
(csrc/conv_stem.hip) and the transparent NCHW -> channels-last routing of paddle.nn.functional
conv2d / batch_norm / max_pool2d, each against a plain PyTorch fp32 reference; the default NCHW
resnet50() must run without a single MIOpen kernel."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
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


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('N,H,W,C,k,s,p,d', [
    (4, 28, 28, 64, 3, 1, 1, 1), (2, 29, 31, 96, 3, 2, 1, 1), (2, 14, 14, 40, 5, 1, 2, 1),
    (2, 17, 17, 32, 7, 2, 3, 1), (2, 20, 20, 48, 3, 1, 2, 2), (1, 9, 9, 1024, 3, 1, 1, 1)])
@pytest.mark.parametrize('bias', [False, True])
def test_dwconv_fwd_bwd(dt, N, H, W, C, k, s, p, d, bias):
    from paddle.ops import conv
    x = torch.randn(N, H, W, C, device=DEV, dtype=dt)
    w = (0.3 * torch.randn(C, 1, k, k, device=DEV)).to(dt)
    b = (0.1 * torch.randn(C, device=DEV)).to(dt) if bias else None
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    yr = torch.nn.functional.conv2d(xr, wr, br, s, p, d, groups=C).permute(0, 2, 3, 1)
    xh, wh = x.clone().requires_grad_(), w.clone().requires_grad_()
    bh = b.clone().requires_grad_() if bias else None
    y = conv.dwconv2d_nhwc(xh, wh, bh, (s, s), (p, p), (d, d))
    assert y.shape == yr.shape
    _close(y, yr, 3e-2, 1e-2, 'dw fwd')
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _close(xh.grad, xr.grad.permute(0, 2, 3, 1), 3e-2, 1e-2, 'dw dgrad')
    _close(wh.grad, wr.grad, 5e-2, 2e-2, 'dw wgrad')
    if bias:
        _close(bh.grad, br.grad, 5e-2, 2e-2, 'dw dbias')


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('N,H,W,C,Cout,k,s,p', [
    (2, 64, 64, 3, 64, 7, 2, 3), (2, 224, 224, 3, 64, 7, 2, 3), (3, 33, 45, 4, 128, 3, 1, 1),
    (2, 40, 40, 1, 64, 5, 2, 2), (1, 300, 300, 3, 64, 3, 2, 1), (2, 96, 96, 3, 32, 3, 2, 1),
    (2, 50, 52, 3, 80, 3, 2, 1),
    # deep filters on the streamed-filter instantiation: AlexNet's 11x11/4 stem (Kp 448), a 9x9 (Kp 288)
    (2, 224, 224, 3, 64, 11, 4, 2), (2, 67, 61, 3, 96, 11, 4, 2), (2, 41, 37, 3, 48, 9, 2, 4),
    # C_out off the 16-channel grain (ShuffleNet v2's 3 -> 24 stem): zero filter rows, sliced output
    (2, 64, 64, 3, 24, 3, 2, 1), (2, 30, 30, 3, 8, 5, 1, 2)])
@pytest.mark.parametrize('bias', [False, True])
def test_conv_stem_fwd(dt, N, H, W, C, Cout, k, s, p, bias):
    from paddle.ops import conv
    x = torch.randn(N, H, W, C, device=DEV, dtype=dt)
    w = (0.2 * torch.randn(Cout, C, k, k, device=DEV)).to(dt)
    b = (0.1 * torch.randn(Cout, device=DEV)).to(dt) if bias else None
    assert conv.stem_ok(x, w, (s, s), (1, 1))
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None if b is None else b.float(), s,
                                     p).permute(0, 2, 3, 1)
    y = conv.conv2d_fwd_stem(x, w, b, (s, s), (p, p))
    assert y.shape == ref.shape
    _close(y, ref, 3e-2, 1e-2, 'stem fwd')


@pytest.mark.parametrize('N,H,W,C,Cout,k,s,p', [
    (2, 224, 224, 3, 64, 7, 2, 3), (3, 64, 64, 3, 64, 7, 2, 3), (2, 33, 45, 4, 128, 3, 1, 1),
    (1, 512, 512, 3, 64, 7, 2, 3), (2, 96, 96, 3, 32, 3, 2, 1), (2, 224, 224, 3, 64, 11, 4, 2)])
def test_conv_stem_bn_stats(N, H, W, C, Cout, k, s, p):
    """Under fused_bn_stats() the stem epilogue's slab (mean, M2) merge to the batch statistics of
    the fp32 convolution (one slab per output-row segment)."""
    from paddle.ops import conv
    x = torch.randn(N, H, W, C, device=DEV).bfloat16()
    w = (0.2 * torch.randn(Cout, C, k, k, device=DEV)).bfloat16()
    with conv.fused_bn_stats():
        y = conv.conv2d_fwd_stem(x, w, None, (s, s), (p, p))
        e = conv.take_bn_parts(y)
    assert e is not None
    parts, P, rpb = e
    M = y.numel() // Cout
    assert P * rpb == M
    pm, pq = parts.view(2, P, Cout)
    mean = pm.mean(0)  # equal slabs
    m2 = pq.sum(0) + rpb * ((pm - mean) ** 2).sum(0)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, s, p).permute(0, 2, 3, 1)
    ref = ref.reshape(M, Cout)
    _close(mean, ref.mean(0), 1e-3, 1e-3, 'stem bn mean')
    _close(m2 / M, ref.var(0, unbiased=False), 1e-3, 1e-2, 'stem bn var')
    _close(y, ref.view_as(y), 3e-2, 1e-2, 'stem fwd (stats launch)')


@pytest.mark.parametrize('C,Cout,k,s,p', [(32, 32, 3, 1, 1), (32, 64, 3, 2, 1), (96, 32, 3, 2, 1), (32, 32, 5, 1, 2)])
def test_conv_zero_tap_padding(C, Cout, k, s, p):
    """K = taps * C an odd multiple of 32 (3x3 over 32 channels): forward and stride-1 / strided
    data gradients run the implicit-GEMM kernels with a zero tap appended; fp32 torch reference,
    and no library convolution kernel in forward + backward."""
    from paddle.ops import conv
    x = torch.randn(2, 19, 21, C, device=DEV).bfloat16()
    w = (0.1 * torch.randn(Cout, C, k, k, device=DEV)).bfloat16()
    assert conv.supported(x, w, 1) and conv.fwd_ok(w)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.float().requires_grad_()
    yr = torch.nn.functional.conv2d(xr, wr, None, s, p).permute(0, 2, 3, 1)
    xh, wh = x.clone().requires_grad_(), w.clone().requires_grad_()
    g = torch.randn_like(yr)

    def run():
        y = conv.conv2d_nhwc(xh, wh, None, (s, s), (p, p), (1, 1))
        y.backward(g.bfloat16())
        return y
    bad = _miopen_kernels(run)
    assert bad == [], bad
    xh.grad = wh.grad = None
    y = run()
    yr.backward(g)
    _close(y, yr, 3e-2, 1e-2, 'fwd')
    _close(xh.grad, xr.grad.permute(0, 2, 3, 1), 3e-2, 1e-2, 'dgrad')
    _close(wh.grad, wr.grad, 5e-2, 2e-2, 'wgrad')


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('N,H,W,C,Cout,G,k,s,p', [
    (2, 14, 14, 128, 128, 32, 3, 1, 1), (2, 15, 13, 256, 256, 32, 3, 2, 1), (1, 9, 9, 1024, 1024, 32, 3, 1, 1),
    (2, 12, 12, 96, 48, 3, 1, 1, 0), (2, 10, 11, 64, 128, 8, 5, 1, 2)])
@pytest.mark.parametrize('bias', [False, True])
def test_gconv_fwd_bwd(dt, N, H, W, C, Cout, G, k, s, p, bias):
    """Grouped conv (csrc/gconv.hip) vs fp32 torch: forward, data and filter gradients (and bias)."""
    from paddle.ops import conv
    x = torch.randn(N, H, W, C, device=DEV, dtype=dt)
    w = (0.2 * torch.randn(Cout, C // G, k, k, device=DEV)).to(dt)
    b = (0.1 * torch.randn(Cout, device=DEV)).to(dt) if bias else None
    assert conv.gconv_supported(x, w, G, (s, s), (p, p), (1, 1))
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    yr = torch.nn.functional.conv2d(xr, wr, br, s, p, 1, groups=G).permute(0, 2, 3, 1)
    xh, wh = x.clone().requires_grad_(), w.clone().requires_grad_()
    bh = b.clone().requires_grad_() if bias else None
    y = conv.gconv2d_nhwc(xh, wh, bh, G, (s, s), (p, p), (1, 1))
    assert y.shape == yr.shape
    _close(y, yr, 3e-2, 1e-2, 'gconv fwd')
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _close(xh.grad, xr.grad.permute(0, 2, 3, 1), 3e-2, 1e-2, 'gconv dgrad')
    _close(wh.grad, wr.grad, 5e-2, 2e-2, 'gconv wgrad')
    if bias:
        _close(bh.grad, br.grad, 5e-2, 2e-2, 'gconv dbias')


def test_resnext_block_nchw_no_miopen():
    """paddle.nn.functional.conv2d with groups=32 (ResNeXt's grouped 3x3) on NCHW bf16: routed to
    the grouped kernels, no library convolution kernel forward or backward."""
    F = paddle.nn.functional
    x = paddle.to_tensor(torch.randn(4, 128, 16, 16, device=DEV).bfloat16())
    x.stop_gradient = False
    w = paddle.to_tensor((0.1 * torch.randn(128, 4, 3, 3, device=DEV)).bfloat16())
    w.stop_gradient = False

    def run():
        y = F.conv2d(x, w, padding=1, groups=32)
        y.sum().backward()
    assert _miopen_kernels(run) == []


@pytest.mark.parametrize('C,Cout,k,s,p', [(24, 144, 1, 1, 0), (144, 24, 1, 1, 0), (16, 96, 1, 1, 0),
                                         (24, 64, 3, 1, 1), (40, 32, 3, 1, 1), (72, 48, 1, 1, 0)])
def test_conv_channel_padding(C, Cout, k, s, p):
    """Input channels C % 32 != 0 (C % 8 == 0, MobileNet pointwise / 3x3 convs): the implicit-GEMM
    forward pads the K decomposition to 32 channels (zero-block chunks x zero filter columns);
    forward, data and filter gradients vs fp32 torch, no library convolution kernel."""
    from paddle.ops import conv
    x = torch.randn(2, 15, 17, C, device=DEV).bfloat16()
    w = (0.1 * torch.randn(Cout, C, k, k, device=DEV)).bfloat16()
    assert conv.supported(x, w, 1) and conv.fwd_ok(w)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.float().requires_grad_()
    yr = torch.nn.functional.conv2d(xr, wr, None, s, p).permute(0, 2, 3, 1)
    xh, wh = x.clone().requires_grad_(), w.clone().requires_grad_()
    g = torch.randn_like(yr)

    def run():
        y = conv.conv2d_nhwc(xh, wh, None, (s, s), (p, p), (1, 1))
        y.backward(g.bfloat16())
        return y
    bad = _miopen_kernels(run)
    assert bad == [], bad
    xh.grad = wh.grad = None
    y = run()
    yr.backward(g)
    _close(y, yr, 3e-2, 1e-2, 'fwd')
    _close(xh.grad, xr.grad.permute(0, 2, 3, 1), 3e-2, 1e-2, 'dgrad')
    _close(wh.grad, wr.grad, 5e-2, 2e-2, 'wgrad')


def _miopen_kernels(fn):
    """Names of the library (MIOpen) convolution / batch-norm / pooling kernels ``fn`` launches."""
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
    bad = ('miopen', 'igemm', 'naive_conv', 'batchnorm', 'im2col', 'col2im', 'conv_fwd', 'conv_bwd', 'gridwise',
           'winograd', 'pooling', 'xdlops', 'subsample', 'sp3asm', 'mlo')
    ours = ('pa::', 'pa_')
    return sorted(n for n in names if any(b in n.lower() for b in bad) and not any(o in n for o in ours))


def test_nchw_conv_bn_pool_routed():
    """NCHW conv2d / batch_norm / max_pool2d on bf16 GPU tensors run the channels-last kernels:
    outputs are NCHW views with channels-last strides, values match fp32 torch, and the profiler
    sees no library convolution kernels."""
    F = paddle.nn.functional
    x = torch.randn(4, 64, 20, 20, device=DEV).bfloat16()
    w = (0.1 * torch.randn(64, 64, 3, 3, device=DEV)).bfloat16()
    gamma = torch.ones(64, device=DEV)
    beta = torch.zeros(64, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    out = {}

    def run():
        y = F.conv2d(paddle.to_tensor(x), paddle.to_tensor(w), padding=1)
        z = F.batch_norm(y, paddle.to_tensor(rm), paddle.to_tensor(rv), paddle.to_tensor(gamma),
                         paddle.to_tensor(beta), training=True)
        out['y'], out['z'] = y._t, z._t
        out['p'] = F.max_pool2d(z, 3, 2, 1)._t

    assert _miopen_kernels(run) == []
    y, z, pool = out['y'], out['z'], out['p']
    assert y.shape == (4, 64, 20, 20) and y.is_contiguous(memory_format=torch.channels_last)
    yr = torch.nn.functional.conv2d(x.float(), w.float(), None, 1, 1)
    _close(y, yr, 3e-2, 1e-2, 'nchw conv')
    zr = torch.nn.functional.batch_norm(yr, None, None, gamma, beta, True, 0.1, 1e-5)
    _close(z, zr, 5e-2, 2e-2, 'nchw bn')
    _close(pool, torch.nn.functional.max_pool2d(z.float(), 3, 2, 1), 1e-6, 0, 'nchw pool')


def test_nchw_depthwise_routed():
    F = paddle.nn.functional
    x = torch.randn(2, 64, 16, 16, device=DEV).bfloat16()
    w = (0.3 * torch.randn(64, 1, 3, 3, device=DEV)).bfloat16()
    out = {}

    def run():
        out['y'] = F.conv2d(paddle.to_tensor(x), paddle.to_tensor(w), stride=2, padding=1, groups=64)._t

    assert _miopen_kernels(run) == []
    ref = torch.nn.functional.conv2d(x.float(), w.float(), None, 2, 1, groups=64)
    _close(out['y'], ref, 3e-2, 1e-2, 'nchw dw')


def test_resnet50_nchw_default_no_miopen():
    """paddle.vision.models.resnet50() with its default data_format='NCHW', AMP-O2 bf16 training
    step: no MIOpen kernel in forward + backward, and the loss equals the NHWC model's with the
    same weights (same kernels, only the layout bookkeeping differs)."""
    from paddle.vision.models import resnet50
    losses = {}
    for df in ('NCHW', 'NHWC'):
        paddle.seed(7)
        net = resnet50(num_classes=10, data_format=df)
        opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=net.parameters(),
                                        multi_precision=True)
        net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
        g = torch.Generator(device=DEV).manual_seed(3)
        img = torch.randn(4, 3, 64, 64, device=DEV, generator=g).bfloat16()
        lab = torch.randint(0, 10, (4,), device=DEV, generator=g)
        xin = paddle.to_tensor(img if df == 'NCHW' else img.permute(0, 2, 3, 1).contiguous())
        y = paddle.to_tensor(lab)
        vals = []

        def step():
            loss = paddle.nn.functional.cross_entropy(net(xin), y)
            loss.backward()
            opt.step()
            opt.clear_grad()
            vals.append(float(loss))

        step()  # warm-up (first-call packing / plans)
        if df == 'NCHW':
            bad = _miopen_kernels(step)
            assert bad == [], bad
        else:
            step()
        losses[df] = vals
    assert all(v == v for v in losses['NCHW'])
    for a, b in zip(losses['NCHW'], losses['NHWC']):
        assert abs(a - b) <= 2e-2 * abs(b) + 1e-3, losses


@pytest.mark.parametrize('N,Cin,Cout,H,k,s,p,op,cl', [
    (2, 64, 32, 9, 4, 2, 1, 0, False), (2, 128, 64, 7, 3, 2, 1, 1, False), (1, 64, 64, 12, 3, 1, 1, 0, True),
    (2, 256, 128, 5, 2, 2, 0, 0, False)])
def test_conv_transpose2d_routed(N, Cin, Cout, H, k, s, p, op, cl):
    """conv2d_transpose on the stride-class data-gradient kernel: forward and all three gradients
    vs fp32 torch, no MIOpen kernels."""
    F = paddle.nn.functional
    x = torch.randn(N, Cin, H, H + 1, device=DEV).bfloat16()
    w = (0.1 * torch.randn(Cin, Cout, k, k, device=DEV)).bfloat16()
    b = (0.1 * torch.randn(Cout, device=DEV)).bfloat16()
    xs = x.permute(0, 2, 3, 1).contiguous() if cl else x
    xp, wp, bp = (paddle.to_tensor(t.clone()) for t in (xs, w, b))
    for t in (xp, wp, bp):
        t.stop_gradient = False
    out = {}

    def run():
        y = F.conv2d_transpose(xp, wp, bp, stride=s, padding=p, output_padding=op,
                               data_format='NHWC' if cl else 'NCHW')
        out['y'] = y
        (y * y).sum().backward()

    assert _miopen_kernels(run) == []
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv_transpose2d(xr, wr, br, s, p, op)
    (yr * yr).sum().backward()
    y = out['y']._t
    _close(y.permute(0, 3, 1, 2) if cl else y, yr, 5e-2, 1e-2, 'convT fwd')
    gx = xp.grad._t
    _close(gx.permute(0, 3, 1, 2) if cl else gx, xr.grad, 0.3, 3e-2, 'convT dx')
    _close(wp.grad._t, wr.grad, 0.5, 3e-2, 'convT dw')
    _close(bp.grad._t, br.grad, 0.5, 3e-2, 'convT db')


@pytest.mark.parametrize('cl', [False, True])
def test_conv1d_routed(cl):
    F = paddle.nn.functional
    x = torch.randn(4, 64, 50, device=DEV).bfloat16()
    w = (0.1 * torch.randn(128, 64, 3, device=DEV)).bfloat16()
    xs = x.permute(0, 2, 1).contiguous() if cl else x
    out = {}

    def run():
        out['y'] = F.conv1d(paddle.to_tensor(xs), paddle.to_tensor(w), padding=1, stride=2,
                            data_format='NLC' if cl else 'NCL')._t

    assert _miopen_kernels(run) == []
    ref = torch.nn.functional.conv1d(x.float(), w.float(), None, 2, 1)
    y = out['y']
    _close(y.permute(0, 2, 1) if cl else y, ref, 3e-2, 1e-2, 'conv1d')


def test_resnext50_nchw_training_step_no_miopen():
    """paddle.vision.models.resnext50_32x4d() (default NCHW, grouped 3x3 convolutions with 4..32
    channels per group) trains an AMP-O2 bf16 step with no library convolution / batch-norm /
    pooling kernel, and its loss is finite."""
    from paddle.vision.models import resnext50_32x4d
    paddle.seed(5)
    net = resnext50_32x4d(num_classes=10)
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=net.parameters(),
                                    multi_precision=True)
    net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
    g = torch.Generator(device=DEV).manual_seed(3)
    xin = paddle.to_tensor(torch.randn(2, 3, 64, 64, device=DEV, generator=g).bfloat16())
    y = paddle.to_tensor(torch.randint(0, 10, (2,), device=DEV, generator=g))
    vals = []

    def step():
        loss = paddle.nn.functional.cross_entropy(net(xin), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        vals.append(float(loss))

    step()
    bad = _miopen_kernels(step)
    assert bad == [], bad
    assert all(v == v and abs(v) < 1e4 for v in vals), vals


def test_mobilenet_v2_nchw_training_step_no_miopen():
    """paddle.vision.models.mobilenet_v2() (default NCHW: 3 -> 32 stem, depthwise 3x3, pointwise
    convs over 16 / 24 / 144 / ... channels) trains an AMP-O2 bf16 step with no library
    convolution / batch-norm / pooling kernel, and its loss is finite."""
    from paddle.vision.models import mobilenet_v2
    paddle.seed(5)
    net = mobilenet_v2(num_classes=10)
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=net.parameters(),
                                    multi_precision=True)
    net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
    g = torch.Generator(device=DEV).manual_seed(3)
    xin = paddle.to_tensor(torch.randn(2, 3, 96, 96, device=DEV, generator=g).bfloat16())
    y = paddle.to_tensor(torch.randint(0, 10, (2,), device=DEV, generator=g))
    vals = []

    def step():
        loss = paddle.nn.functional.cross_entropy(net(xin), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        vals.append(float(loss))

    step()
    bad = _miopen_kernels(step)
    assert bad == [], bad
    assert all(v == v and abs(v) < 1e4 for v in vals), vals


@pytest.mark.parametrize('C', [58, 116, 3])
def test_bn_channel_pad_matches_torch(C):
    """Batch norm over a channel count off the 16-byte grain runs the HIP kernels on a zero-padded
    copy: output, input / gamma / beta gradients and running statistics match the fp32 reference."""
    from paddle.ops import batchnorm as BN
    g = torch.Generator(device=DEV).manual_seed(C)
    x = torch.randn(4, 7, 9, C, device=DEV, generator=g).bfloat16().requires_grad_()
    gam = (torch.rand(C, device=DEV, generator=g) + 0.5).requires_grad_()
    bet = torch.randn(C, device=DEV, generator=g).requires_grad_()
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    assert not BN.supported(x, gam) and BN.channel_pad_ok(x, gam)
    y = BN.bn_nhwc_cpad(x, gam, bet, rm, rv, 1e-5, 0.9, True)
    dy = torch.randn(y.shape, device=DEV, generator=g).bfloat16()
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    gr, br = gam.detach().clone().requires_grad_(), bet.detach().clone().requires_grad_()
    rmr, rvr = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yr = torch.nn.functional.batch_norm(xr, rmr, rvr, gr, br, True, 0.1, 1e-5)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert y.shape == x.shape
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=6e-2, rtol=3e-2)
    torch.testing.assert_close(gam.grad, gr.grad, atol=5e-1, rtol=2e-2)
    torch.testing.assert_close(bet.grad, br.grad, atol=5e-1, rtol=2e-2)
    torch.testing.assert_close(rm, rmr, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(rv, rvr, atol=2e-3, rtol=2e-3)



@pytest.mark.parametrize('C,Cout,k,p,bias', [(512, 10, 1, 0, True), (64, 10, 3, 1, False), (128, 3, 3, 1, True)])
def test_conv_cout_padding(C, Cout, k, p, bias):
    """C_out % 8 != 0 (SqueezeNet's 10-class 1x1 head): paddle.nn.functional.conv2d pads C_out with
    zero filters onto the implicit-GEMM kernels and slices the output; forward, data / filter / bias
    gradients vs fp32 torch, no library convolution kernel."""
    F = paddle.nn.functional
    x = torch.randn(2, C, 13, 15, device=DEV).bfloat16()
    w = (0.05 * torch.randn(Cout, C, k, k, device=DEV)).bfloat16()
    b = torch.randn(Cout, device=DEV).bfloat16() if bias else None
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    br = b.float().requires_grad_() if bias else None
    yr = torch.nn.functional.conv2d(xr, wr, br, 1, p)
    g = torch.randn_like(yr)
    xp = paddle.to_tensor(x, stop_gradient=False)
    wp = paddle.to_tensor(w, stop_gradient=False)
    bp = paddle.to_tensor(b, stop_gradient=False) if bias else None
    out = []

    def run():
        y = F.conv2d(xp, wp, bp, 1, p)
        y.backward(paddle.to_tensor(g.bfloat16()))
        out.append(y)
    bad = _miopen_kernels(run)
    assert bad == [], bad
    yr.backward(g)
    y = out[0]._t if hasattr(out[0], '_t') else out[0]
    assert tuple(y.shape) == tuple(yr.shape)
    _close(y, yr, 3e-2, 1e-2, 'fwd')
    _close(xp.grad._t, xr.grad, 3e-2, 1e-2, 'dgrad')
    _close(wp.grad._t, wr.grad, 5e-2, 2e-2, 'wgrad')
    if bias:
        _close(bp.grad._t, br.grad, 5e-2, 2e-2, 'bgrad')


@pytest.mark.parametrize('C,Cout,k,s,p,groups', [(58, 58, 1, 1, 0, 1), (116, 232, 1, 1, 0, 1), (58, 64, 3, 2, 1, 1),
                                                  (58, 58, 3, 1, 1, 58), (58, 58, 3, 2, 1, 58), (116, 116, 3, 2, 1, 116)])
def test_conv_cin_padding(C, Cout, k, s, p, groups):
    """C_in % 8 != 0 (ShuffleNet v2's 58 / 116-channel branches): plain and depthwise conv2d run on
    the hand-written kernels over a zero-padded channels-last copy; forward, data / filter / bias
    gradients vs fp32 torch, no library convolution kernel."""
    F = paddle.nn.functional
    x = torch.randn(2, C, 14, 13, device=DEV).bfloat16()
    w = (0.1 * torch.randn(Cout, C // groups, k, k, device=DEV)).bfloat16()
    b = torch.randn(Cout, device=DEV).bfloat16()
    xr, wr, br = (v.float().requires_grad_() for v in (x, w, b))
    yr = torch.nn.functional.conv2d(xr, wr, br, s, p, 1, groups)
    g = torch.randn_like(yr)
    xp, wp, bp = (paddle.to_tensor(v, stop_gradient=False) for v in (x, w, b))
    out = []

    def run():
        y = F.conv2d(xp, wp, bp, s, p, groups=groups)
        y.backward(paddle.to_tensor(g.bfloat16()))
        out.append(y)
    bad = _miopen_kernels(run)
    assert bad == [], bad
    yr.backward(g)
    y = out[0]._t
    assert tuple(y.shape) == tuple(yr.shape)
    _close(y, yr, 3e-2, 1e-2, 'fwd')
    _close(xp.grad._t, xr.grad, 3e-2, 1e-2, 'dgrad')
    _close(wp.grad._t, wr.grad, 5e-2, 2e-2, 'wgrad')
    _close(bp.grad._t, br.grad, 5e-2, 2e-2, 'bgrad')


@pytest.mark.parametrize('C,Cout,D,k,s,p,fmt', [(32, 64, 8, 3, 1, 1, 'NCDHW'), (64, 32, 9, 3, 2, 1, 'NCDHW'),
                                               (16, 32, 6, 1, 1, 0, 'NDHWC'), (32, 32, 7, 3, 1, 0, 'NDHWC')])
def test_conv3d_depth_taps_on_hip_kernels(C, Cout, D, k, s, p, fmt):
    """conv3d folded onto the 2-D implicit-GEMM kernels (one batched 2-D convolution per depth tap):
    forward, data / filter / bias gradients vs fp32 torch, no library convolution kernel."""
    F = paddle.nn.functional
    x = torch.randn(2, C, D, 10, 12, device=DEV).bfloat16()
    w = (0.05 * torch.randn(Cout, C, k, k, k, device=DEV)).bfloat16()
    b = torch.randn(Cout, device=DEV).bfloat16()
    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv3d(xr, wr, br, s, p)
    g = torch.randn_like(yr)
    xin = x if fmt == 'NCDHW' else x.permute(0, 2, 3, 4, 1).contiguous()
    xp = paddle.to_tensor(xin, stop_gradient=False)
    wp = paddle.to_tensor(w, stop_gradient=False)
    bp = paddle.to_tensor(b, stop_gradient=False)
    out = []

    def run():
        y = F.conv3d(xp, wp, bp, s, p, data_format=fmt)
        gg = g if fmt == 'NCDHW' else g.permute(0, 2, 3, 4, 1)
        y.backward(paddle.to_tensor(gg.bfloat16().contiguous()))
        out.append(y)
    bad = _miopen_kernels(run)
    assert bad == [], bad
    yr.backward(g)
    y = out[0]._t
    if fmt == 'NDHWC':
        y = y.permute(0, 4, 1, 2, 3)
    assert tuple(y.shape) == tuple(yr.shape)
    _close(y, yr, 3e-2, 1e-2, 'fwd')
    dx = xp.grad._t if fmt == 'NCDHW' else xp.grad._t.permute(0, 4, 1, 2, 3)
    _close(dx, xr.grad, 3e-2, 1e-2, 'dgrad')
    _close(wp.grad._t, wr.grad, 5e-2, 2e-2, 'wgrad')
    _close(bp.grad._t, br.grad, 5e-2, 2e-2, 'bgrad')


@pytest.mark.parametrize('C,Cout,D,k,s,p,op', [(32, 64, 4, 3, 1, 1, 0), (64, 32, 5, 3, 2, 1, 1), (32, 32, 4, 2, 2, 0, 0)])
def test_conv3d_transpose_depth_taps_on_hip_kernels(C, Cout, D, k, s, p, op):
    """conv3d_transpose folded onto the 2-D transposed-conv kernels (one batched transposed 2-D
    convolution per depth tap, slices index-added into the output depth): forward, data / filter /
    bias gradients vs fp32 torch, no library convolution kernel."""
    F = paddle.nn.functional
    x = torch.randn(2, C, D, 8, 9, device=DEV).bfloat16()
    w = (0.05 * torch.randn(C, Cout, k, k, k, device=DEV)).bfloat16()
    b = torch.randn(Cout, device=DEV).bfloat16()
    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv_transpose3d(xr, wr, br, s, p, op)
    g = torch.randn_like(yr)
    xp = paddle.to_tensor(x, stop_gradient=False)
    wp = paddle.to_tensor(w, stop_gradient=False)
    bp = paddle.to_tensor(b, stop_gradient=False)
    out = []

    def run():
        y = F.conv3d_transpose(xp, wp, bp, s, p, output_padding=op)
        y.backward(paddle.to_tensor(g.bfloat16().contiguous()))
        out.append(y)
    bad = _miopen_kernels(run)
    assert bad == [], bad
    yr.backward(g)
    y = out[0]._t
    assert tuple(y.shape) == tuple(yr.shape)
    _close(y, yr, 3e-2, 1e-2, 'fwd')
    _close(xp.grad._t, xr.grad, 3e-2, 1e-2, 'dgrad')
    _close(wp.grad._t, wr.grad, 5e-2, 2e-2, 'wgrad')
    _close(bp.grad._t, br.grad, 5e-2, 2e-2, 'bgrad')
