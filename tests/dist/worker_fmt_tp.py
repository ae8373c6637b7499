"""fused_multi_transformer with ring_id (2 gloo ranks): each rank holds half of the heads / FFN
columns; the out-linear and ffn2 partial outputs are all-reduced over the ring group.  Must equal
the unsharded call (reference: incubate/nn/functional/fused_transformer.py:964, ring_id)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.incubate.nn.functional as IF  # noqa: E402


def main():
    dist.init_parallel_env()
    r, W = dist.get_rank(), dist.get_world_size()
    g = dist.new_group(list(range(W)))
    B, S, E, H, F = 2, 5, 32, 4, 64
    D = E // H
    gen = torch.Generator().manual_seed(3)
    rnd = lambda *s: torch.randn(*s, generator=gen) * 0.2  # noqa: E731
    full = dict(ln_scales=[torch.ones(E)], ln_biases=[torch.zeros(E)], qkv_weights=[rnd(3, H, D, E)],
                qkv_biases=[rnd(3 * H * D)], linear_weights=[rnd(H * D, E)], linear_biases=[rnd(E)],
                ffn_ln_scales=[torch.ones(E)], ffn_ln_biases=[torch.zeros(E)], ffn1_weights=[rnd(E, F)],
                ffn1_biases=[rnd(F)], ffn2_weights=[rnd(F, E)], ffn2_biases=[rnd(E)])
    x = rnd(B, S, E)
    hs, fs = slice(r * H // W, (r + 1) * H // W), slice(r * F // W, (r + 1) * F // W)
    part = dict(full)
    part['qkv_weights'] = [full['qkv_weights'][0][:, hs].contiguous()]
    part['qkv_biases'] = [full['qkv_biases'][0].reshape(3, H, D)[:, hs].reshape(-1).contiguous()]
    part['linear_weights'] = [full['linear_weights'][0][hs.start * D:hs.stop * D].contiguous()]
    part['ffn1_weights'] = [full['ffn1_weights'][0][:, fs].contiguous()]
    part['ffn1_biases'] = [full['ffn1_biases'][0][fs].contiguous()]
    part['ffn2_weights'] = [full['ffn2_weights'][0][fs].contiguous()]
    t = paddle.to_tensor
    wrap = lambda d: {k: [t(v) for v in vs] for k, vs in d.items()}  # noqa: E731
    want = IF.fused_multi_transformer(t(x), **wrap(full))
    got = IF.fused_multi_transformer(t(x), ring_id=g.id, **wrap(part))
    np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=1e-4, atol=1e-5)
    # fused_feedforward / fused_multi_head_attention (training path): outputs and input gradients
    w1, b1, w2, b2 = rnd(E, F), rnd(F), rnd(F, E), rnd(E)
    xf = t(x)
    xf.stop_gradient = False
    ref = IF.fused_feedforward(xf, t(w1), t(w2), t(b1), t(b2), dropout1_rate=0.0, dropout2_rate=0.0)
    ref.sum().backward()
    gref = xf.grad.numpy().copy()
    xp = t(x)
    xp.stop_gradient = False
    out = IF.fused_feedforward(xp, t(w1[:, fs].contiguous()), t(w2[fs].contiguous()), t(b1[fs].contiguous()), t(b2),
                               dropout1_rate=0.0, dropout2_rate=0.0, ring_id=g.id)
    out.sum().backward()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(xp.grad.numpy(), gref, rtol=1e-4, atol=1e-5)
    qw, qb, lw, lb = rnd(3, H, D, E), rnd(3 * H * D), rnd(H * D, E), rnd(E)
    xa = t(x)
    xa.stop_gradient = False
    ref = IF.fused_multi_head_attention(xa, t(qw), t(lw), qkv_bias=t(qb), linear_bias=t(lb), dropout_rate=0.0,
                                        attn_dropout_rate=0.0)
    ref.sum().backward()
    xb = t(x)
    xb.stop_gradient = False
    out = IF.fused_multi_head_attention(xb, t(qw[:, hs].contiguous()), t(lw[hs.start * D:hs.stop * D].contiguous()),
                                        qkv_bias=t(qb.reshape(3, H, D)[:, hs].reshape(-1).contiguous()),
                                        linear_bias=t(lb), dropout_rate=0.0, attn_dropout_rate=0.0, ring_id=g.id)
    out.sum().backward()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(xb.grad.numpy(), xa.grad.numpy(), rtol=1e-4, atol=1e-5)
    print(f"rank{r} fmt tp OK", flush=True)
    dist.barrier()


if __name__ == '__main__':
    main()
