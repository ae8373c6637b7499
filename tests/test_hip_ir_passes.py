"""IR fusion passes on the GPU: a static ERNIE program (AMP-O2 bf16) run by the Executor with the
fused nodes (flash attention with the padding mask and in-kernel dropout, fused add + LayerNorm on
csrc/norm.hip) vs the same program unfused (fusion off: the recorded torch ops)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
from paddle import static  # noqa: E402
from paddle.static import ir_passes as IP  # noqa: E402
from paddle.ops import flash_attn as FA, norm as NORM, fused as FUSED, matmul as HM  # noqa: E402

from test_ir_passes import _build, _feed  # noqa: E402


def _run(train, drop, mode, steps=3):
    old = IP.set_mode(mode)
    try:
        paddle.set_device('gpu:0')
        paddle.seed(5)
        main, loss, logits = _build(train, drop, hidden=128, heads=2)
        static.amp.cast_model_to_fp16(main, dest_type='bfloat16', level='O1')  # autocast replay
        paddle.enable_static()
        try:
            exe = static.Executor(paddle.CUDAPlace(0))
            outs = [exe.run(main, feed=_feed(), fetch_list=[loss, logits]) for _ in range(steps)]
        finally:
            paddle.disable_static()
        return outs, IP.fusion_stats(main)
    finally:
        IP.set_mode(old)


class _Count:
    def __init__(self, mod, name):
        self.mod, self.name, self.n = mod, name, 0

    def __enter__(self):
        self.orig = getattr(self.mod, self.name)

        def f(*a, **k):
            self.n += 1
            return self.orig(*a, **k)
        setattr(self.mod, self.name, f)
        return self

    def __exit__(self, *a):
        setattr(self.mod, self.name, self.orig)


def test_ernie_static_fused_kernels_match_unfused_program():
    ref, _ = _run(False, 0.0, '0', steps=1)
    with _Count(FA, 'flash_attention_packed_ex') as ca, _Count(NORM, 'add_layer_norm') as cn:
        out, stats = _run(False, 0.0, 'auto', steps=1)
    assert stats.get('multihead_matmul_fuse_pass_v2') == 2, stats  # packed q / k / v slices of the qkv GEMM
    # 4 of the 5 add + LayerNorm sites: the embedding sum stays fp32 under O1 autocast (embedding
    # lookups are not autocast ops), so that one takes the composite
    assert ca.n == 2 and cn.n == 4, (ca.n, cn.n)
    np.testing.assert_allclose(out[0][1], ref[0][1], rtol=5e-2, atol=5e-2)
    np.testing.assert_allclose(out[0][0], ref[0][0], rtol=3e-2, atol=3e-2)


def test_ernie_static_amp_bf16_training_fused():
    """AMP-O2 bf16 training with dropout: the fused program takes the flash kernel (mask + dropout),
    the fused dropout + add + LayerNorm kernels and the GELU-epilogue FFN op, and trains (finite,
    decreasing loss)."""
    old = IP.set_mode('auto')
    try:
        paddle.set_device('gpu:0')
        paddle.seed(5)
        paddle.enable_static()
        try:
            from paddle.models import ernie_config, ErnieForSequenceClassification
            cfg = ernie_config('ernie-tiny', hidden_size=128, num_attention_heads=2)
            main, startup = static.Program(), static.Program()
            with static.program_guard(main, startup):
                ids = static.data('ids', [None, 32], 'int64')
                lab = static.data('lab', [None], 'int64')
                model = ErnieForSequenceClassification(cfg, num_classes=2)
                loss = paddle.nn.functional.cross_entropy(model(ids), lab)
                opt = static.amp.decorate(paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters()),
                                          level='O2', dtype='bfloat16')
                opt.minimize(loss)
            exe = static.Executor(paddle.CUDAPlace(0))
            opt.amp_init(paddle.CUDAPlace(0))
            with _Count(FA, 'flash_attention_packed_ex') as ca, _Count(FUSED, 'dropout_add_norm') as cd, \
                    _Count(HM, 'ffn_gelu') as cf:
                losses = [float(np.asarray(exe.run(main, feed=_feed(), fetch_list=[loss])[0]).reshape(-1)[0])
                          for _ in range(8)]
        finally:
            paddle.disable_static()
    finally:
        IP.set_mode(old)
    assert ca.n == 16 and cd.n == 32 and cf.n == 16, (ca.n, cd.n, cf.n)  # cf: GELU FFNs in the GEMM epilogues
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
    assert torch.cuda.is_available()


def test_programdesc_predictor_bf16_fused_vs_unfused(tmp_path):
    """An ERNIE ProgramDesc run by the bf16 Predictor with the IR passes (flash attention, fused
    add + LayerNorm, GEMM + bias) vs the same model with switch_ir_optim(False)."""
    from paddle import inference as I
    from test_ir_passes import _ernie_inference_model
    prefix, feed, _ = _ernie_inference_model(tmp_path)

    def pred(ir):
        c = I.Config(prefix + '.pdmodel', prefix + '.pdiparams')
        c.enable_use_gpu(256, 0, I.PrecisionType.Bfloat16)
        c.switch_ir_optim(ir)
        return I.create_predictor(c)
    x = paddle.to_tensor(feed, place=paddle.CUDAPlace(0))
    ref = pred(False).run([x])[0].numpy()
    p = pred(True)
    with _Count(FA, 'flash_attention_ex') as ca, _Count(NORM, 'add_layer_norm') as cn:
        out = p.run([x])[0].numpy()
    assert IP.fusion_stats(p._program).get('multihead_matmul_fuse_pass_v2') == 2
    assert ca.n == 2 and cn.n == 5, (ca.n, cn.n)
    np.testing.assert_allclose(out, ref, rtol=5e-2, atol=5e-2)


def test_resnet50_predictor_folds_batch_norm_gpu():
    """ResNet50 inference program (bf16, NCHW) on the Executor: conv2d_bn_fuse_pass folds every
    batch norm into its convolution, conv2d_add_act_fuse_pass takes the residual adds and ReLUs, and
    the convolutions run on the hand-written kernels — the profiler sees no batch-norm kernel and no
    library convolution; the output matches the unfused program."""
    from test_hip_conv_routing import _miopen_kernels
    paddle.set_device('gpu:0')
    paddle.seed(2)
    paddle.enable_static()
    try:
        main, st = static.Program(), static.Program()
        with static.program_guard(main, st):
            x = static.data('x', [None, 3, 64, 64], 'bfloat16')
            m = paddle.vision.models.resnet50(num_classes=100)
            m.to(dtype='bfloat16')
            m.eval()
            y = m(x)
    finally:
        paddle.disable_static()
    xv = paddle.to_tensor(np.random.RandomState(0).randn(8, 3, 64, 64).astype('float32')).astype('bfloat16')

    def run(mode):
        old = IP.set_mode(mode)
        paddle.enable_static()
        try:
            return static.Executor(paddle.CUDAPlace(0)).run(main, feed={'x': xv}, fetch_list=[y],
                                                            return_numpy=False)[0]._t.float()
        finally:
            paddle.disable_static()
            IP.set_mode(old)
    ref = run('0')
    got = run('auto')
    st = IP.fusion_stats(main)
    assert st.get('conv2d_bn_fuse_pass') == 53, st
    assert st.get('conv2d_add_act_fuse_pass', 0) >= 49, st
    err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-3)
    assert err < 5e-2, err
    bad = [n for n in _miopen_kernels(lambda: run('auto')) if 'batchnorm' in n.lower() or 'conv' in n.lower()
           or 'igemm' in n.lower() or 'xdlops' in n.lower()]
    assert bad == [], bad


def test_fused_bn_add_act_pass_static_training_gpu():
    """A recorded conv -> BN -> ReLU / conv -> BN -> +residual -> ReLU training program on the GPU:
    the fused_bn_add_act_pass nodes run the HIP batch-norm kernels (statistics, apply, residual, ReLU
    in one autograd op) and three SGD steps equal the unfused (library) program."""
    from test_ir_passes_ext import _bn_block_program
    from paddle.ops import batchnorm as BN
    calls = []
    orig = BN.bn_act_nhwc

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    rng = np.random.RandomState(0)
    batches = [(rng.randn(32, 8, 6, 6).astype('float32'), rng.randint(0, 8, (32,)).astype("int64"))
               for _ in range(3)]
    paddle.set_device('gpu')
    paddle.enable_static()
    res = []
    try:
        for fused in (False, True):
            main, startup, loss = _bn_block_program()
            main._ir_passes = ['fused_bn_add_act_pass'] if fused else []
            exe = static.Executor(paddle.CUDAPlace(0))
            exe.run(startup)
            BN.bn_act_nhwc = counting
            try:
                ls = [float(exe.run(main, feed={'x': xb, 'y': yb}, fetch_list=[loss])[0]) for xb, yb in batches]
            finally:
                BN.bn_act_nhwc = orig
            res.append((ls, [p.numpy().copy() for p in main.all_parameters()]))
            if fused:
                assert main._ir_stats.get('fused_bn_add_act_pass') == 2, main._ir_stats
                assert len(calls) == 2 * len(batches)
            else:
                assert not calls
    finally:
        paddle.disable_static()
        paddle.set_device('cpu')
    np.testing.assert_allclose(res[0][0], res[1][0], rtol=1e-4, atol=1e-5)
    for a, b in zip(res[0][1], res[1][1]):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-4)
