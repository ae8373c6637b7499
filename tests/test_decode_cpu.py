"""Decode-phase attention APIs on CPU (torch reference paths; the HIP kernels are compared against
the same references in tests/test_hip_kernels.py): masked_multihead_attention,
block_multihead_attention over a paged cache, fused_multi_transformer / FusedMultiTransformer
incremental decoding == full-sequence forward."""
import math

import numpy as np
import pytest
import torch

import paddle
import paddle.incubate.nn.functional as IF
from paddle.incubate.nn import FusedMultiTransformer
from paddle.ops import decode


def _attn(q, k, v, causal=True):
    """q [S, H, D], k/v [L, Hkv, D] -> [S, H, D] (bottom-right causal)."""
    S, H, D = q.shape
    L, Hkv = k.shape[0], k.shape[1]
    k = k.repeat_interleave(H // Hkv, 1)
    v = v.repeat_interleave(H // Hkv, 1)
    s = torch.einsum('shd,lhd->hsl', q.double(), k.double()) / math.sqrt(D)
    if causal:
        i = torch.arange(S)[:, None] + (L - S)
        s = s.masked_fill(torch.arange(L)[None, :] > i, float('-inf'))
    return torch.einsum('hsl,lhd->shd', torch.softmax(s, -1), v.double())


def test_masked_multihead_attention_matches_reference():
    torch.manual_seed(0)
    B, H, L, D = 3, 4, 32, 16
    cache = torch.randn(2, B, H, L, D)
    x = torch.randn(B, 3 * H * D)
    bias = torch.randn(3, H, D) * 0.1
    steps = torch.tensor([[5], [0], [17]])
    want_cache = cache.clone()
    out, c = IF.masked_multihead_attention(paddle.to_tensor(x), paddle.to_tensor(cache), bias=paddle.to_tensor(bias),
                                           sequence_lengths=paddle.to_tensor(steps))
    qkv = x.reshape(B, 3, H, D) + bias
    for b in range(B):
        t = int(steps[b])
        want_cache[0, b, :, t] = qkv[b, 1]
        want_cache[1, b, :, t] = qkv[b, 2]
        o = _attn(qkv[b, 0][None], want_cache[0, b, :, :t + 1].transpose(0, 1), want_cache[1, b, :, :t + 1].transpose(0, 1),
                  causal=False)[0]
        np.testing.assert_allclose(out.numpy()[b], o.reshape(-1).numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(c.numpy(), want_cache.numpy(), atol=1e-6)


def test_decode_attention_paged_equals_contiguous():
    torch.manual_seed(1)
    B, Hq, Hkv, D, bs = 2, 4, 2, 8, 4
    L = 12
    kc = torch.randn(B, Hkv, L, D)
    vc = torch.randn(B, Hkv, L, D)
    nblk = B * L // bs
    perm = torch.randperm(nblk)
    bt = perm.reshape(B, L // bs)
    kp = torch.empty(nblk, Hkv, bs, D)
    vp = torch.empty(nblk, Hkv, bs, D)
    for b in range(B):
        for j in range(L // bs):
            kp[bt[b, j]] = kc[b, :, j * bs:(j + 1) * bs]
            vp[bt[b, j]] = vc[b, :, j * bs:(j + 1) * bs]
    q = torch.randn(B, Hq, D)
    lens = torch.tensor([7, 12])
    a = decode.decode_attention(q, kc, vc, lens)
    p = decode.decode_attention(q, kp, vp, lens, block_tables=bt)
    np.testing.assert_allclose(a.numpy(), p.numpy(), rtol=1e-5, atol=1e-6)


def test_decode_attention_int8_cache_matches_dequantised():
    """8-bit caches (int8 / uint8 with zero point 128; static [Hkv] and per-sequence [B, Hkv]
    dequant scales, paged and contiguous) == attention over the dequantised bf16 / fp32 cache."""
    torch.manual_seed(3)
    B, Hq, Hkv, D, bs, L = 2, 4, 2, 8, 4, 12
    for cdt, zp in ((torch.int8, 0), (torch.uint8, 128)):
        for dyn in (False, True):
            kq = torch.randint(-127, 128, (B, Hkv, L, D))
            vq = torch.randint(-127, 128, (B, Hkv, L, D))
            ks = torch.rand((B, Hkv) if dyn else (Hkv,)) * 0.05 + 0.01
            vs = torch.rand((B, Hkv) if dyn else (Hkv,)) * 0.05 + 0.01
            q = torch.randn(B, Hq, D)
            lens = torch.tensor([5, 12])
            kd = kq.float() * ks.reshape(-1, Hkv)[:, :, None, None]
            vd = vq.float() * vs.reshape(-1, Hkv)[:, :, None, None]
            want = decode.decode_attention_ref(q, kd.expand(B, -1, -1, -1), vd.expand(B, -1, -1, -1), lens)
            got = decode.decode_attention(q, (kq + zp).to(cdt), (vq + zp).to(cdt), lens, k_dequant=ks, v_dequant=vs)
            np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=1e-5, atol=1e-6)
            nblk = B * L // bs
            bt = torch.randperm(nblk).reshape(B, L // bs)
            kp = torch.empty(nblk, Hkv, bs, D, dtype=cdt)
            vp = torch.empty(nblk, Hkv, bs, D, dtype=cdt)
            for b in range(B):
                for j in range(L // bs):
                    kp[bt[b, j]] = (kq[b, :, j * bs:(j + 1) * bs] + zp).to(cdt)
                    vp[bt[b, j]] = (vq[b, :, j * bs:(j + 1) * bs] + zp).to(cdt)
            got = decode.decode_attention(q, kp, vp, lens, block_tables=bt, k_dequant=ks, v_dequant=vs)
            np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=1e-5, atol=1e-6)


def _get_padding_offset(this):
    cu = torch.zeros(len(this) + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(torch.tensor(this), 0)
    return cu


def test_block_multihead_attention_mixed_batch():
    """two prompts (prefill into their blocks) + two decode tokens over their cached prefixes"""
    torch.manual_seed(2)
    Hq, Hkv, D, bs, nblk = 4, 2, 8, 4, 24
    kc = torch.zeros(nblk, Hkv, bs, D)
    vc = torch.zeros(nblk, Hkv, bs, D)
    enc = [5, 0, 3, 0]
    dec = [0, 6, 0, 9]
    this = [5, 1, 3, 1]
    bt = torch.arange(nblk).reshape(4, 6)
    # pre-fill the decode sequences' prefixes
    hist = {1: (torch.randn(6, Hkv, D), torch.randn(6, Hkv, D)), 3: (torch.randn(9, Hkv, D), torch.randn(9, Hkv, D))}
    for b, (k, v) in hist.items():
        for p in range(k.shape[0]):
            kc[bt[b, p // bs], :, p % bs] = k[p]
            vc[bt[b, p // bs], :, p % bs] = v[p]
    T = sum(this)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D)
    cu = _get_padding_offset(this)
    out, _, kc2, vc2 = IF.block_multihead_attention(
        paddle.to_tensor(qkv), paddle.to_tensor(kc), paddle.to_tensor(vc),
        paddle.to_tensor(torch.tensor(enc)[:, None]), paddle.to_tensor(torch.tensor(dec)[:, None]),
        paddle.to_tensor(torch.tensor(this)[:, None]), None, None, paddle.to_tensor(cu), paddle.to_tensor(cu),
        paddle.to_tensor(bt), block_size=bs)
    o = out.numpy()
    for b in range(4):
        s0, n = int(cu[b]), this[b]
        rows = qkv[s0:s0 + n]
        q = rows[:, :Hq * D].reshape(n, Hq, D)
        k = rows[:, Hq * D:(Hq + Hkv) * D].reshape(n, Hkv, D)
        v = rows[:, (Hq + Hkv) * D:].reshape(n, Hkv, D)
        if b in hist:
            k = torch.cat([hist[b][0], k])
            v = torch.cat([hist[b][1], v])
        want = _attn(q, k, v, causal=True)
        np.testing.assert_allclose(o[s0:s0 + n], want.reshape(n, -1).numpy(), rtol=1e-4, atol=1e-5)
        # the new tokens' K/V are in the cache at their positions
        p_last = dec[b] + n - 1
        np.testing.assert_allclose(kc2.numpy()[bt[b, p_last // bs], :, p_last % bs], k[-1].numpy(), atol=1e-6)


@pytest.mark.parametrize("gqa", [-1, 2])
@pytest.mark.parametrize("norm", ['layernorm', 'rmsnorm'])
def test_fused_multi_transformer_incremental_decode(gqa, norm):
    paddle.seed(3)
    E, H, F_, nl, B, S, Lmax = 32, 4, 64, 2, 2, 6, 16
    m = FusedMultiTransformer(E, H, F_, num_layers=nl, norm_type=norm, gqa_group_size=gqa)
    m.eval()
    Hkv = gqa if gqa > 0 else H
    D = E // H
    x = paddle.randn([B, S + 2, E])
    full = m(x)  # causal forward over all S+2 positions (no cache)
    caches = [paddle.zeros([2, B, Hkv, Lmax, D]) for _ in range(nl)]
    out, caches = m(x[:, :S], caches=caches)
    np.testing.assert_allclose(out.numpy(), full.numpy()[:, :S], rtol=1e-4, atol=1e-5)
    for t in range(S, S + 2):
        o, caches = m(x[:, t:t + 1], caches=caches, time_step=paddle.to_tensor([t]))
        np.testing.assert_allclose(o.numpy()[:, 0], full.numpy()[:, t], rtol=1e-4, atol=1e-5)


def test_fused_multi_transformer_functional_reference_shapes():
    paddle.seed(4)
    E, H, D = 16, 2, 8
    x = paddle.randn([2, 3, E])
    args = dict(ln_scales=[paddle.ones([E])], ln_biases=[paddle.zeros([E])],
                qkv_weights=[paddle.randn([3, H, D, E]) * 0.1], qkv_biases=[paddle.zeros([3, H, D])],
                linear_weights=[paddle.randn([E, E]) * 0.1], linear_biases=[paddle.zeros([E])],
                ffn_ln_scales=[paddle.ones([E])], ffn_ln_biases=[paddle.zeros([E])],
                ffn1_weights=[paddle.randn([E, 4 * E]) * 0.1], ffn1_biases=[paddle.zeros([4 * E])],
                ffn2_weights=[paddle.randn([4 * E, E]) * 0.1], ffn2_biases=[paddle.zeros([E])])
    out = IF.fused_multi_transformer(x, **args)
    assert list(out.shape) == [2, 3, E]
    mask = paddle.zeros([2, 1, 3, 3])
    out2 = IF.fused_multi_transformer(x, attn_mask=mask, **args)  # explicit (non-causal) mask
    assert not np.allclose(out.numpy(), out2.numpy())


def _mmha_inputs(B, H, L, D, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 3 * H * D, generator=g)
    cache = torch.randn(2, B, H, L, D, generator=g)
    return x, cache


def test_mmha_beam_cache_offset_matches_rearranged_cache():
    """beam_cache_offset: each beam reads past positions from the cache row of its ancestor beam."""
    import paddle
    import paddle.incubate.nn.functional as IF
    B, beam, H, L, D, t = 4, 2, 2, 8, 16, 5
    x, cache = _mmha_inputs(B, H, L, D, 0)
    off = torch.randint(0, beam, (B // beam, beam, L), generator=torch.Generator().manual_seed(1))
    seq = torch.full((B, 1), t, dtype=torch.int32)
    c1 = cache.clone()
    out, c1o, off_out = IF.masked_multihead_attention(paddle.to_tensor(x), paddle.to_tensor(c1),
                                                      sequence_lengths=paddle.to_tensor(seq),
                                                      beam_cache_offset=paddle.to_tensor(off))
    # reference: rearrange every row's past positions explicitly, then the plain decode step
    c2 = cache.clone()
    for b in range(B):
        for p in range(t):
            src = (b // beam) * beam + int(off[b // beam, b % beam, p])
            c2[:, b, :, p] = cache[:, src, :, p]
    ref, _ = IF.masked_multihead_attention(paddle.to_tensor(x), paddle.to_tensor(c2),
                                           sequence_lengths=paddle.to_tensor(seq))
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    assert off_out is not None


def test_mmha_quant_paths():
    """qkv_out_scale dequantises an int32 qkv; out_scale quantises the output (round half away)."""
    import paddle
    import paddle.incubate.nn.functional as IF
    B, H, L, D, t = 2, 2, 8, 16, 3
    g = torch.Generator().manual_seed(2)
    xi = torch.randint(-500, 500, (B, 3 * H * D), generator=g, dtype=torch.int32)
    sc = torch.rand(3, H, D, generator=g) * 0.01
    _, cache = _mmha_inputs(B, H, L, D, 3)
    seq = paddle.to_tensor(torch.full((B, 1), t, dtype=torch.int32))
    o1, _ = IF.masked_multihead_attention(paddle.to_tensor(xi), paddle.to_tensor(cache.clone()), sequence_lengths=seq,
                                          qkv_out_scale=paddle.to_tensor(sc), compute_dtype='fp32')
    xf = xi.float() * sc.reshape(1, -1)
    o2, _ = IF.masked_multihead_attention(paddle.to_tensor(xf), paddle.to_tensor(cache.clone()), sequence_lengths=seq)
    np.testing.assert_allclose(o1.numpy(), o2.numpy(), rtol=1e-5, atol=1e-6)
    oq, _ = IF.masked_multihead_attention(paddle.to_tensor(xf), paddle.to_tensor(cache.clone()), sequence_lengths=seq,
                                          out_scale=0.5, quant_round_type=1)
    v = o2.numpy() * 127.0 * 0.5
    expect = np.clip(np.sign(v) * np.floor(np.abs(v) + 0.5), -127, 127).astype(np.int8)
    assert oq.numpy().dtype == np.int8
    np.testing.assert_array_equal(oq.numpy(), expect)


def test_fused_multi_transformer_pre_caches_decode():
    """A pre-cache prefix is attended to ahead of the cached sequence: identical to placing the
    prefix at the start of the cache and decoding P steps later (no rotary embedding)."""
    import paddle
    import paddle.incubate.nn.functional as IF
    B, S0, E, H, P, L = 2, 3, 32, 2, 4, 16
    D = E // H
    g = torch.Generator().manual_seed(4)
    t = paddle.to_tensor
    w = lambda *s: t(torch.randn(*s, generator=g) * 0.2)  # noqa: E731
    params = dict(ln_scales=[t(torch.ones(E))], ln_biases=[t(torch.zeros(E))], qkv_weights=[w(3, H, D, E)],
                  qkv_biases=[w(3 * H * D)], linear_weights=[w(E, E)], linear_biases=[w(E)],
                  ffn_ln_scales=[t(torch.ones(E))], ffn_ln_biases=[t(torch.zeros(E))], ffn1_weights=[w(E, 2 * E)],
                  ffn1_biases=[w(2 * E)], ffn2_weights=[w(2 * E, E)], ffn2_biases=[w(E)])
    x = w(B, 1, E)
    pre = torch.randn(2, B, H, P, D, generator=g)
    hist = torch.randn(2, B, H, L, D, generator=g)
    c1 = hist.clone()
    c1[:, :, :, S0 + 1:] = 0
    o1, _ = IF.fused_multi_transformer(x, cache_kvs=[t(c1)], pre_caches=[t(pre)], time_step=t(torch.tensor([S0])),
                                       **params)
    c2 = torch.zeros(2, B, H, L + P, D)
    c2[:, :, :, :P] = pre
    c2[:, :, :, P:P + S0] = hist[:, :, :, :S0]
    o2, _ = IF.fused_multi_transformer(x, cache_kvs=[t(c2)], time_step=t(torch.tensor([S0 + P])), **params)
    np.testing.assert_allclose(o1.numpy(), o2.numpy(), rtol=1e-4, atol=1e-5)


def _blha_case(seed, quant=False, pre=0):
    torch.manual_seed(seed)
    Hq, Hkv, D, bs, nblk = 4, 2, 8, 4, 24
    dt = torch.int8 if quant else torch.float32
    kc = torch.zeros(nblk, Hkv, bs, D, dtype=dt)
    vc = torch.zeros(nblk, Hkv, bs, D, dtype=dt)
    enc, dec, this = [5, 0, 3, 0], [0, 6, 0, 9], [5, 1, 3, 1]
    bt = torch.arange(nblk).reshape(4, 6)
    qs = torch.tensor([20.0, 30.0])           # quant scales per kv head
    dq = 1.0 / qs
    qz = lambda x: torch.clamp(torch.sign(x * qs[None, :, None]) *  # noqa: E731
                               torch.floor((x * qs[None, :, None]).abs() + 0.5), -127, 127)
    hist = {1: (torch.randn(6, Hkv, D), torch.randn(6, Hkv, D)), 3: (torch.randn(9, Hkv, D), torch.randn(9, Hkv, D))}
    for b, (k, v) in hist.items():
        for p in range(k.shape[0]):
            kc[bt[b, p // bs], :, p % bs] = (qz(k[p:p + 1])[0] if quant else k[p]).to(dt)
            vc[bt[b, p // bs], :, p % bs] = (qz(v[p:p + 1])[0] if quant else v[p]).to(dt)
    T = sum(this)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D)
    cu = _get_padding_offset(this)
    pk = torch.randn(4, Hkv, pre, D) if pre else None
    pv = torch.randn(4, Hkv, pre, D) if pre else None
    t = paddle.to_tensor
    kw = {}
    if quant:
        kw = dict(cache_k_quant_scales=t(qs), cache_v_quant_scales=t(qs), cache_k_dequant_scales=t(dq),
                  cache_v_dequant_scales=t(dq))
    if pre:
        kw.update(pre_key_cache=t(pk), pre_value_cache=t(pv))
    out, _, kc2, _ = IF.block_multihead_attention(
        t(qkv), t(kc), t(vc), t(torch.tensor(enc)[:, None]), t(torch.tensor(dec)[:, None]),
        t(torch.tensor(this)[:, None]), None, None, t(cu), t(cu), t(bt), block_size=bs, **kw)
    o = out.numpy()
    for b in range(4):
        s0, n = int(cu[b]), this[b]
        rows = qkv[s0:s0 + n]
        q = rows[:, :Hq * D].reshape(n, Hq, D)
        k = rows[:, Hq * D:(Hq + Hkv) * D].reshape(n, Hkv, D)
        v = rows[:, (Hq + Hkv) * D:].reshape(n, Hkv, D)
        if b in hist:  # decode rows read everything (incl. their new K/V) back from the cache
            hk, hv = hist[b]
            if quant:
                hk, hv = qz(hk) * dq[None, :, None], qz(hv) * dq[None, :, None]
                k, v = qz(k) * dq[None, :, None], qz(v) * dq[None, :, None]
            k, v = torch.cat([hk, k]), torch.cat([hv, v])
        if pre:
            k, v = torch.cat([pk[b].permute(1, 0, 2), k]), torch.cat([pv[b].permute(1, 0, 2), v])
        want = _attn(q, k, v, causal=True)
        np.testing.assert_allclose(o[s0:s0 + n], want.reshape(n, -1).numpy(), rtol=1e-4, atol=1e-4)
    return kc2


def test_block_multihead_attention_pre_caches():
    """A per-sequence prefix (pre_key/value_cache) ahead of prompts and decode rows."""
    _blha_case(5, pre=3)


def test_block_multihead_attention_int8_cache():
    """Static int8 KV cache: new rows quantised into the pages, decode reads dequantised pages."""
    kc2 = _blha_case(6, quant=True)
    assert kc2.numpy().dtype == np.int8
    _blha_case(7, quant=True, pre=2)


def test_block_multihead_attention_dynamic_uint8_cache():
    """Dynamic KV-cache quantisation into uint8 pages (value + 128): a prompt step writes
    per-(sequence, head) scales max_bound / absmax, a decode step reuses them."""
    torch.manual_seed(8)
    Hq, Hkv, D, bs, nblk, B = 2, 2, 8, 4, 8, 2
    t = paddle.to_tensor
    kc = torch.zeros(nblk, Hkv, bs, D, dtype=torch.uint8)
    vc = torch.zeros(nblk, Hkv, bs, D, dtype=torch.uint8)
    bt = torch.arange(nblk).reshape(B, 4)
    scales = [torch.zeros(B, Hkv) for _ in range(4)]
    kw = dict(cache_k_quant_scales=t(scales[0]), cache_v_quant_scales=t(scales[1]),
              cache_k_dequant_scales=t(scales[2]), cache_v_dequant_scales=t(scales[3]),
              use_dynamic_cachekv_quant=True)
    # step 1: sequence 0 is a 5-token prompt, sequence 1 idle
    qkv1 = torch.randn(5, (Hq + 2 * Hkv) * D)
    cu1 = _get_padding_offset([5, 0])
    _, _, kc_t, vc_t = IF.block_multihead_attention(
        t(qkv1), t(kc), t(vc), t(torch.tensor([[5], [0]])), t(torch.tensor([[0], [0]])), t(torch.tensor([[5], [0]])),
        None, None, t(cu1), t(cu1), t(bt), block_size=bs, **kw)
    k1 = qkv1[:, Hq * D:(Hq + Hkv) * D].reshape(5, Hkv, D)
    v1 = qkv1[:, (Hq + Hkv) * D:].reshape(5, Hkv, D)
    amax_k, amax_v = k1.abs().amax(dim=(0, 2)), v1.abs().amax(dim=(0, 2))
    np.testing.assert_allclose(kw['cache_k_quant_scales'].numpy()[0], (127.0 / amax_k).numpy(), rtol=1e-6)
    np.testing.assert_allclose(kw['cache_v_dequant_scales'].numpy()[0], (amax_v / 127.0).numpy(), rtol=1e-6)
    assert (kw['cache_k_quant_scales'].numpy()[1] == 0).all()  # the idle sequence keeps its scales
    kq = kc_t.numpy()[bt[0, 0], :, 0].astype(np.float32) - 128.0
    np.testing.assert_allclose(kq * (amax_k / 127.0).numpy()[:, None], k1[0].numpy(), atol=float(amax_k.max()) / 127)
    # step 2: sequence 0 decodes its 6th token against the dequantised prompt
    qkv2 = torch.randn(1, (Hq + 2 * Hkv) * D)
    cu2 = _get_padding_offset([1, 0])
    out, _, _, _ = IF.block_multihead_attention(
        t(qkv2), kc_t, vc_t, t(torch.tensor([[0], [0]])), t(torch.tensor([[5], [0]])), t(torch.tensor([[1], [0]])),
        None, None, t(cu2), t(cu2), t(bt), block_size=bs, **kw)
    qs_k, qs_v = 127.0 / amax_k, 127.0 / amax_v

    def rt(x, s):  # quantise then dequantise, round half away from zero
        return torch.clamp(torch.sign(x * s[None, :, None]) * torch.floor((x * s[None, :, None]).abs() + 0.5),
                           -127, 127) / s[None, :, None]
    k2 = qkv2[:, Hq * D:(Hq + Hkv) * D].reshape(1, Hkv, D)
    v2 = qkv2[:, (Hq + Hkv) * D:].reshape(1, Hkv, D)
    kk = torch.cat([rt(k1, qs_k), rt(k2, qs_k)])
    vv = torch.cat([rt(v1, qs_v), rt(v2, qs_v)])
    want = _attn(qkv2[:, :Hq * D].reshape(1, Hq, D), kk, vv, causal=False)
    np.testing.assert_allclose(out.numpy(), want.reshape(1, -1).numpy(), rtol=1e-4, atol=1e-4)
