"""Real RCCL collectives on one GPU: a 1-rank ``nccl`` process group with
PADDLE_AMD_FORCE_COLLECTIVES=1 disables every world-1 short-circuit of the sharding / DP engines,
so the all-gather / reduce-scatter / all-reduce calls, their streams and their ordering against the
in-place HIP weight-gradient GEMMs (grouped / deferred wgrads included) run exactly as on 8 GPUs.
A 1-rank AVG / SUM is the identity, so the result must match the aliased (no-collective) path."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
import torch.distributed as dist  # noqa: E402

DEV = 'cuda'


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope='module')
def nccl_world1():
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(_port())
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    assert dist.get_backend() == 'nccl'
    yield
    dist.destroy_process_group()


def _gpt_run(force, level, steps=3):
    from paddle.models.gpt import gpt_config, GPTForPretraining
    os.environ['PADDLE_AMD_FORCE_COLLECTIVES'] = '1' if force else '0'
    try:
        paddle.seed(0)
        cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        model = GPTForPretraining(cfg)
        opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters(), multi_precision=True,
                                     grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
        model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
        model, opt, _ = paddle.distributed.sharding.group_sharded_parallel(model, opt, level=level)
        eng = opt.engine
        assert eng.collectives == force and eng.alias == (not force)
        ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (4, 129), device=DEV,
                                             generator=torch.Generator(device=DEV).manual_seed(1)))
        x, y = ids[:, :-1], ids[:, 1:]
        inner = model._layers if hasattr(model, '_layers') else model
        losses = []
        for _ in range(steps):
            loss = inner.loss(model(x), y)
            loss.backward()
            opt.step()
            opt.clear_grad()
            losses.append(float(loss))
        eng.wait_param_gathers()
        params = [torch.cat([eng.pshard(u).float() for u in eng.units])]
        return losses, params
    finally:
        os.environ['PADDLE_AMD_FORCE_COLLECTIVES'] = '0'


@pytest.mark.parametrize('level', ['p_g_os', 'os_g', 'os'])
def test_sharding_real_rccl_matches_alias(nccl_world1, level):
    la, pa = _gpt_run(False, level)
    lf, pf = _gpt_run(True, level)
    assert all(l == l for l in lf)
    for a, b in zip(la, lf):
        assert abs(a - b) <= 1e-6 * abs(a), (la, lf)
    for a, b in zip(pa, pf):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5), float((a - b).abs().max())


def test_data_parallel_real_rccl(nccl_world1):
    """DataParallel over a 1-rank RCCL group (bucketed async all-reduce from the grad-ready hooks)
    on a conv net: same parameters as the plain model after a few Momentum steps."""
    nn = paddle.nn
    finals = []
    for force in (False, True):
        os.environ['PADDLE_AMD_FORCE_COLLECTIVES'] = '1' if force else '0'
        try:
            paddle.seed(3)
            net = nn.Sequential(nn.Conv2D(16, 32, 3, padding=1, data_format='NHWC'), nn.BatchNorm2D(32, data_format='NHWC'),
                                nn.ReLU(), nn.AdaptiveAvgPool2D(1, data_format='NHWC'), nn.Flatten(), nn.Linear(32, 10))
            opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=net.parameters(),
                                            multi_precision=True)
            net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
            dp = paddle.DataParallel(net)
            assert (dp._reducer is not None) == force
            g = torch.Generator(device=DEV).manual_seed(4)
            x = paddle.to_tensor(torch.randn(8, 16, 16, 16, device=DEV, generator=g).bfloat16())
            y = paddle.to_tensor(torch.randint(0, 10, (8,), device=DEV, generator=g))
            for _ in range(3):
                loss = paddle.nn.functional.cross_entropy(dp(x), y)
                loss.backward()
                opt.step()
                opt.clear_grad()
            finals.append([p._t.float().clone() for p in net.parameters()])
        finally:
            os.environ['PADDLE_AMD_FORCE_COLLECTIVES'] = '0'
    for a, b in zip(*finals):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5), float((a - b).abs().max())
