"""Sharding offload on the GPU (world 1): the optimizer state of the shard in pinned host memory,
the step's D2H gradient copy, the host-runtime AdamW (csrc/runtime pa_rt_adamw) and the H2D
parameter copy must reproduce plain on-device AdamW; bf16 parameters keep fp32 masters on the host."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402


def _net(seed=3):
    paddle.seed(seed)
    return paddle.nn.Sequential(paddle.nn.Linear(64, 256), paddle.nn.GELU(), paddle.nn.Linear(256, 64))


@pytest.mark.parametrize('level', ['os_g', 'p_g_os'])
def test_offload_adamw_matches_device_adamw(level):
    paddle.set_device('gpu:0')
    ref, net = _net(), _net()
    ropt = paddle.optimizer.AdamW(1e-2, parameters=ref.parameters(), weight_decay=0.05)
    opt = paddle.optimizer.AdamW(1e-2, parameters=net.parameters(), weight_decay=0.05)
    model, sopt, _ = paddle.distributed.sharding.group_sharded_parallel(net, opt, level=level, offload=True)
    eng = model._engine
    assert all(a['m'].device.type == 'cpu' and a['m'].is_pinned() for a in eng.arenas.values())
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        x = paddle.to_tensor(torch.randn(32, 64, generator=g).cuda())
        for m, o in ((ref, ropt), (model, sopt)):
            loss = (m(x) ** 2).mean()
            loss.backward()
            o.step()
            o.clear_grad()
    sd = model.state_dict()
    for k, v in ref.state_dict().items():
        np.testing.assert_allclose(sd[k].numpy(), v.numpy(), rtol=2e-5, atol=2e-6, err_msg=k)


def test_offload_bf16_parameters_fp32_host_master():
    paddle.set_device('gpu:0')
    net = _net()
    for p in net.parameters():
        p._t.data = p._t.data.to(torch.bfloat16)
    ref = [p._t.detach().float().clone() for p in net.parameters()]
    opt = paddle.optimizer.AdamW(1e-3, parameters=net.parameters(), weight_decay=0.0)
    model, sopt, _ = paddle.distributed.sharding.group_sharded_parallel(net, opt, level='os_g', offload=True)
    a = next(iter(model._engine.arenas.values()))
    assert a['master'].dtype == torch.float32 and a['master'].device.type == 'cpu'
    x = paddle.to_tensor(torch.randn(16, 64).cuda().to(torch.bfloat16))
    (model(x).astype('float32') ** 2).mean().backward()
    sopt.step()
    sopt.clear_grad()
    # the device bf16 parameters are the rounded host masters
    got = torch.cat([p._t.detach().float().reshape(-1).cpu() for p in net.parameters()])
    master = a['master'][:got.numel()]
    assert torch.equal(got, master.to(torch.bfloat16).float())
    assert not torch.equal(got, torch.cat([r.reshape(-1).cpu() for r in ref]))
