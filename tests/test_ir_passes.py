"""IR fusion passes (static/ir_passes.py): the rewritten program computes what the recorded one
computes.  CPU: fusion forced on ('always'), the fused entry points take their composite paths, so
every output must be bit-identical to the unfused run (same ops, same RNG order) — in eval and over
three AdamW training steps with dropout; the rewrite counts pin what matched.  The GPU half
(kernels inside the fused nodes vs the unfused program) is tests/test_hip_ir_passes.py."""
import numpy as np
import pytest
import torch

import paddle
from paddle import static
from paddle.static import ir_passes as IP
from paddle.models import ernie_config, ErnieForSequenceClassification


_FUSIONS = ('multihead_matmul_fuse_pass_v2', 'skip_layernorm_fuse_pass', 'fused_dropout_add_layernorm',
            'fuse_gemm_epilogue_pass', 'layer_norm_fuse_pass', 'fc_fuse_pass', 'softmax_fuse_pass',
            'quant_linear_fuse_pass', 'embedding_eltwise_layernorm_fuse_pass')


def _build(train, drop, hidden=64, heads=2):
    paddle.seed(5)
    paddle.enable_static()
    try:
        cfg = ernie_config('ernie-tiny', hidden_dropout_prob=drop, attention_probs_dropout_prob=drop,
                           hidden_size=hidden, num_attention_heads=heads)
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            ids = static.data('ids', [None, 32], 'int64')
            lab = static.data('lab', [None], 'int64')
            model = ErnieForSequenceClassification(cfg, num_classes=2)
            if not train:
                model.eval()
            logits = model(ids)
            loss = paddle.nn.functional.cross_entropy(logits, lab)
            if train:
                paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters()).minimize(loss)
    finally:
        paddle.disable_static()
    return main, loss, logits


def _feed():
    rng = np.random.RandomState(0)
    ids = rng.randint(1, 512, size=(4, 32)).astype('int64')
    ids[1, 20:] = 0  # padding: the attention mask is live
    return {'ids': ids, 'lab': rng.randint(0, 2, size=(4,)).astype('int64')}


@pytest.fixture
def fusion_mode():
    old = IP.set_mode('always')
    yield
    IP.set_mode(old)


@pytest.mark.parametrize('train,drop,expect', [
    # inference: the embeddings' sum + LayerNorm is the embedding_eltwise_layernorm_fuse_pass's
    (False, 0.1, {'multihead_matmul_fuse_pass_v2': 2, 'skip_layernorm_fuse_pass': 4, 'fuse_gemm_epilogue_pass': 2,
                  'embedding_eltwise_layernorm_fuse_pass': 1}),
    (True, 0.1, {'multihead_matmul_fuse_pass_v2': 2, 'fused_dropout_add_layernorm': 4, 'skip_layernorm_fuse_pass': 1,
                 'fuse_gemm_epilogue_pass': 2}),
    (True, 0.0, {'multihead_matmul_fuse_pass_v2': 2, 'skip_layernorm_fuse_pass': 5, 'fuse_gemm_epilogue_pass': 2}),
])
def test_ernie_program_fused_equals_unfused(fusion_mode, train, drop, expect):
    feed = _feed()
    res = []
    for mode in ('0', 'always'):
        IP.set_mode(mode)
        paddle.seed(5)
        main, loss, logits = _build(train, drop)
        n_before = len(main.nodes)
        exe = static.Executor(paddle.CPUPlace())
        paddle.seed(7)
        paddle.enable_static()
        try:
            res.append([exe.run(main, feed=feed, fetch_list=[loss, logits]) for _ in range(3)])
        finally:
            paddle.disable_static()
        assert len(main.nodes) == n_before  # the program itself is never rewritten
        if mode == 'always':
            assert {k: v for k, v in IP.fusion_stats(main).items() if k in _FUSIONS} == expect
    for a, b in zip(*res):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


def test_fused_entry_points_composite_semantics():
    import torch
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(2, 3, 5, 8, generator=g) for _ in range(3))
    keep = torch.rand(2, 1, 1, 5, generator=g) > 0.3
    keep[..., 0] = True
    ref = torch.softmax((q @ k.transpose(-1, -2)).float() * 0.3 + torch.where(keep, 0.0, -1e30), -1) @ v
    for mode, m in (('keep', keep), ('drop', ~keep), ('add', torch.where(keep, 0.0, -1e30))):
        out = IP.fused_attention(q, k, v, m, scale=0.3, mask_mode=mode)
        assert torch.allclose(out, ref, atol=1e-5)
    out = IP.fused_attention(q, k.transpose(-1, -2), v, keep, scale=0.3, mask_mode='keep', k_transposed=True)
    assert torch.allclose(out, ref, atol=1e-5)
    x, r = torch.randn(4, 16, generator=g), torch.randn(4, 16, generator=g)
    w, b = torch.randn(16, generator=g), torch.randn(16, generator=g)
    y, s = IP.fused_dropout_add_layer_norm(x, r, w, b, 1e-5, 0.0)
    assert torch.allclose(s, x + r) and torch.allclose(y, torch.nn.functional.layer_norm(x + r, [16], w, b))
    W = torch.randn(16, 8, generator=g)
    assert torch.allclose(IP.fused_linear(x, W, b[:8], 'relu'), torch.relu(x @ W + b[:8]))
    assert torch.allclose(IP.fused_linear(x, W.t().contiguous(), None, 'gelu', trans_w=True),
                          torch.nn.functional.gelu(x @ W), atol=1e-6)


def test_shared_mask_invert_not_claimed(fusion_mode):
    """A mask value used by two attentions: each fuses, the shared invert stays in the program."""
    import torch
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data('x', [2, 2, 4, 8], 'float32')
            m = static.data('m', [2, 1, 1, 4], 'bool')
            inv = ~m._t
            outs = []
            for _ in range(2):
                s = torch.matmul(x._t, x._t.transpose(-1, -2)) * 0.5
                p = torch.softmax(s.masked_fill(inv, -1e30), -1)
                outs.append(torch.matmul(p, x._t))
            _ = outs[0] + outs[1]
    finally:
        paddle.disable_static()
    nodes, stats = IP.apply_passes(main)
    assert stats.get('multihead_matmul_fuse_pass_v2') == 2
    assert any(IP._kind(n) == 'invert' for n in nodes)


def _ernie_inference_model(tmp_path, hidden=128, heads=2):
    import os
    paddle.set_device('cpu')  # the model is built and exported on the CPU (GPU boxes included)
    paddle.seed(0)
    paddle.enable_static()
    try:
        cfg = ernie_config('ernie-tiny', hidden_size=hidden, num_attention_heads=heads)
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            ids = static.data('ids', [None, 32], 'int64')
            model = ErnieForSequenceClassification(cfg, num_classes=2)
            model.eval()
            logits = model(ids)
        exe = static.Executor(paddle.CPUPlace())
        prefix = os.path.join(str(tmp_path), 'ernie')
        static.save_inference_model(prefix, [ids], [logits], exe, program=main)
        feed = _feed()['ids'][:3]
        ref = exe.run(main, feed={'ids': feed}, fetch_list=[logits])[0]
    finally:
        paddle.disable_static()
    return prefix, feed, ref


def test_programdesc_ernie_predictor_fused(tmp_path, fusion_mode):
    """ERNIE exported as a reference ProgramDesc (.pdmodel) and run by the inference Predictor: the
    imported-operator passes (matmul_v2 / scale / where / softmax / matmul_v2 attention, add +
    layer_norm, matmul_v2 + elementwise_add fc) rewrite it, and it computes the recorded program's
    outputs exactly."""
    from paddle import inference as I
    prefix, feed, ref = _ernie_inference_model(tmp_path)
    pred = I.create_predictor(I.Config(prefix + '.pdmodel', prefix + '.pdiparams'))
    assert getattr(pred._program, '_pdmodel', False)  # really the ProgramDesc import
    out = pred.run([paddle.to_tensor(feed)])[0].numpy()
    assert IP.fusion_stats(pred._program) == {'multihead_matmul_fuse_pass_v2': 2, 'skip_layernorm_fuse_pass': 5,
                                              'fc_fuse_pass': 10}
    np.testing.assert_array_equal(out, ref)
    cfg = I.Config(prefix + '.pdmodel', prefix + '.pdiparams')
    cfg.switch_ir_optim(False)
    pred2 = I.create_predictor(cfg)
    np.testing.assert_array_equal(pred2.run([paddle.to_tensor(feed)])[0].numpy(), ref)
    assert IP.fusion_stats(pred2._program) == {}


def test_programdesc_bf16_predictor_casts_parameters(tmp_path):
    """A bf16 Predictor over a ProgramDesc model runs its loaded parameters (resolved through their
    owners) in bf16, so the fused entry points see 16-bit operands."""
    from paddle import inference as I
    prefix, feed, _ = _ernie_inference_model(tmp_path)
    c = I.Config(prefix + '.pdmodel', prefix + '.pdiparams')
    c.enable_use_gpu(256, 0, I.PrecisionType.Bfloat16)
    p = I.create_predictor(c)
    prog = p._program
    owners = prog._const_owner
    assert owners
    for cid, o in owners.items():
        if o._t.is_floating_point():
            assert o._t.dtype == torch.bfloat16 and prog.consts[cid] is o._t
    out = p.run([paddle.to_tensor(feed)])[0]
    assert np.isfinite(out.numpy()).all()
