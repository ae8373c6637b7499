"""General and convolution IR passes (static/ir_passes_ext.py; reference conv2d_bn_fuse_pass.cc,
conv2d_add_act_fuse_pass.cc, constant_folding_pass.cc, dead_code_elimination_pass.cc,
common_subexpression_elimination_pass.cc, fused_weight_only_linear_pass.cc): the rewritten program
computes what the recorded one computes (CPU, fusion forced on)."""
import numpy as np
import pytest
import torch

import paddle
from paddle import static
from paddle.static import ir_passes as IP
from paddle.static import ir_passes_ext as IX


@pytest.fixture
def fusion_mode():
    old = IP.set_mode('always')
    yield
    IP.set_mode(old)


def _run(main, feed, fetch, mode):
    old = IP.set_mode(mode)
    try:
        paddle.enable_static()
        exe = static.Executor(paddle.CPUPlace())
        return exe.run(main, feed=feed, fetch_list=fetch)
    finally:
        paddle.disable_static()
        IP.set_mode(old)


def _resnet_program(arch='resnet18', train=False):
    paddle.seed(1)
    paddle.enable_static()
    try:
        main, st = static.Program(), static.Program()
        with static.program_guard(main, st):
            x = static.data('x', [None, 3, 32, 32], 'float32')
            m = getattr(paddle.vision.models, arch)(num_classes=10)
            # non-trivial running statistics so the fold is exercised
            for layer in m.sublayers():
                if isinstance(layer, paddle.nn.BatchNorm2D):
                    c = layer._mean.shape[0]
                    layer._mean.set_value(np.random.RandomState(c).randn(c).astype('float32') * 0.1)
                    layer._variance.set_value(np.random.RandomState(c + 1).rand(c).astype('float32') + 0.5)
                    layer.weight.set_value(np.random.RandomState(c + 2).rand(c).astype('float32') + 0.5)
                    layer.bias.set_value(np.random.RandomState(c + 3).randn(c).astype('float32') * 0.1)
            m.eval()
            y = m(x)
    finally:
        paddle.disable_static()
    return main, y


def test_conv_bn_fold_and_conv_add_act_resnet18():
    main, y = _resnet_program()
    xv = np.random.RandomState(0).randn(2, 3, 32, 32).astype('float32')
    ref, = _run(main, {'x': xv}, [y], '0')
    got, = _run(main, {'x': xv}, [y], 'always')
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
    st = IP.fusion_stats(main)
    assert st.get('conv2d_bn_fuse_pass') == 20, st          # every conv + BN pair of resnet18
    assert st.get('conv2d_add_act_fuse_pass', 0) >= 16, st  # conv -> relu and conv -> + residual -> relu
    nodes = main._ir_cache[1]
    names = [getattr(n.target, '__name__', '') for n in nodes]
    assert 'batch_norm' not in names and 'relu' not in names  # no standalone BN / ReLU left
    # batch size 5 after the rewrite (the folded program keeps dynamic dims)
    xv5 = np.random.RandomState(1).randn(5, 3, 32, 32).astype('float32')
    np.testing.assert_allclose(_run(main, {'x': xv5}, [y], 'always')[0], _run(main, {'x': xv5}, [y], '0')[0],
                               rtol=1e-4, atol=1e-4)


def test_conv_bn_fold_skipped_for_training_programs(fusion_mode):
    paddle.seed(1)
    paddle.enable_static()
    try:
        main, st = static.Program(), static.Program()
        with static.program_guard(main, st):
            x = static.data('x', [None, 3, 16, 16], 'float32')
            conv = paddle.nn.Conv2D(3, 8, 3, padding=1)
            bn = paddle.nn.BatchNorm2D(8)
            bn.eval()
            loss = paddle.nn.functional.relu(bn(conv(x))).mean()
            paddle.optimizer.SGD(0.1, parameters=conv.parameters()).minimize(loss)
        exe = static.Executor(paddle.CPUPlace())
        exe.run(main, feed={'x': np.ones([2, 3, 16, 16], 'float32')}, fetch_list=[loss])
    finally:
        paddle.disable_static()
    assert 'conv2d_bn_fuse_pass' not in IP.fusion_stats(main)  # weights change: never folded


def test_constant_folding_dce_cse(fusion_mode):
    paddle.enable_static()
    try:
        main, st = static.Program(), static.Program()
        with static.program_guard(main, st):
            x = static.data('x', [None, 4], 'float32')
            a = paddle.tanh(x)
            b = paddle.tanh(x)                # same op, same operand: merged
            dead = paddle.sin(x) * 3.0        # never fetched: dropped
            y0 = a + b
        # a constant-only chain as an imported program carries one (a recorded program folds such
        # chains while it is built): exp(c) * 2 on a captured constant, then added to y0
        from paddle.static.program import Node, Ref, Const
        from paddle.core.tensor import _wrap
        c = Const(main._const(torch.arange(4, dtype=torch.float32)))
        v1, v2, v3 = next(main._vid), next(main._vid), next(main._vid)
        main.nodes += [Node('torch', torch.exp, [c], {}, v1), Node('torch', torch.mul, [Ref(v1), 2.0], {}, v2),
                       Node('torch', torch.add, [Ref(main._val[id(y0._t)]), Ref(v2)], {}, v3)]
        with paddle.static.program._paused():
            ym = torch.empty(0, device='meta')
        main._val[id(ym)] = v3
        main._keep.append(ym)
        y = _wrap(ym)
        exe = static.Executor(paddle.CPUPlace())
        xv = np.random.RandomState(0).randn(3, 4).astype('float32')
        got, = exe.run(main, feed={'x': xv}, fetch_list=[y])
        st = IP.fusion_stats(main)
        # fetching `dead` too (a different fetch set) keeps it
        got2, d2 = exe.run(main, feed={'x': xv}, fetch_list=[y, dead])
    finally:
        paddle.disable_static()
    ref = 2 * np.tanh(xv) + np.exp(np.arange(4)) * 2.0
    np.testing.assert_allclose(got, ref, rtol=1e-5)
    np.testing.assert_allclose(got2, ref, rtol=1e-5)
    np.testing.assert_allclose(d2, np.sin(xv) * 3.0, rtol=1e-5)
    assert st.get('constant_folding_pass', 0) >= 1, st
    assert st.get('common_subexpression_elimination_pass', 0) >= 1, st
    assert st.get('dead_code_elimination_pass', 0) >= 2, st  # sin and its scale


def test_cse_never_merges_random_ops(fusion_mode):
    paddle.enable_static()
    try:
        main, st = static.Program(), static.Program()
        with static.program_guard(main, st):
            x = static.data('x', [None, 64], 'float32')
            a = paddle.nn.functional.dropout(x, 0.5)
            b = paddle.nn.functional.dropout(x, 0.5)
            y = a - b
        exe = static.Executor(paddle.CPUPlace())
        out, = exe.run(main, feed={'x': np.ones([8, 64], 'float32')}, fetch_list=[y])
    finally:
        paddle.disable_static()
    assert np.abs(out).sum() > 0  # two independent masks


def test_weight_only_linear_pass_opt_in(fusion_mode):
    paddle.seed(3)
    paddle.enable_static()
    try:
        main, st = static.Program(), static.Program()
        with static.program_guard(main, st):
            x = static.data('x', [None, 128], 'bfloat16')
            lin = paddle.nn.Linear(128, 64)
            lin.to(dtype='bfloat16')
            y = lin(x)
    finally:
        paddle.disable_static()
    xv = np.random.RandomState(0).randn(4, 128).astype('float32')
    main._ir_passes = IP.DEFAULT_PASSES + ('fused_weight_only_linear_pass',)
    paddle.enable_static()
    try:
        exe = static.Executor(paddle.CPUPlace())
        xt = paddle.to_tensor(xv).astype('bfloat16')
        got, = exe.run(main, feed={'x': xt}, fetch_list=[y])
    finally:
        paddle.disable_static()
    assert IP.fusion_stats(main).get('fused_weight_only_linear_pass') == 1
    w = main.all_parameters()
    W = [p for p in w if p._t.dim() == 2][0]._t.detach().float().numpy()
    B = [p for p in w if p._t.dim() == 1][0]._t.detach().float().numpy()
    want = xt._t.float().numpy() @ W + B
    np.testing.assert_allclose(np.asarray(got, dtype='float32'), want, rtol=0.05, atol=0.05)
    _ = IX


def test_inplace_pass_rewrites_dying_operands_only():
    """inplace_pass: relu / add of a dying fresh operand become in-place; a value that is fetched,
    viewed or read later keeps the out-of-place op; results are unchanged."""
    from paddle.static import ir_passes as IP
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data('x', [4, 8], 'float32')
            lin = paddle.nn.Linear(8, 8)
            h = lin(x)                      # fresh (addmm)
            a = paddle.nn.functional.relu(h)  # h dies here -> in place
            b = a * 2.0                     # a dies -> in place
            v = b.reshape([8, 4])           # b is viewed: the next op must not write into b
            c = paddle.nn.functional.relu(b)
            out = c.sum() + v.sum()
        exe = paddle.static.Executor()
        xv = np.random.RandomState(0).randn(4, 8).astype('float32')
        ref = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
        nodes, stats = IP.apply_passes(main, passes=['inplace_pass'], fetch=(main._val[id(out._t)],))
        assert stats.get('inplace_pass') == 2, stats
        inplace = [n for n in nodes if (n.meta or {}).get('inplace')]
        assert len(inplace) == 2
        main._ir_passes = ['inplace_pass']
        import os
        os.environ['FLAGS_static_ir_fusion'] = '1'
        try:
            IP._MODE[0] = '1'
            got = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
        finally:
            IP._MODE[0] = 'auto'
            os.environ.pop('FLAGS_static_ir_fusion', None)
        np.testing.assert_allclose(got, ref, rtol=1e-6)
    finally:
        paddle.disable_static()


def _bn_block_program(seed=3):
    paddle.seed(seed)
    main, startup = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, startup):
        x = paddle.static.data('x', [-1, 8, 6, 6], 'float32')
        y = paddle.static.data('y', [-1], 'int64')
        c1 = paddle.nn.Conv2D(8, 8, 3, padding=1)
        b1 = paddle.nn.BatchNorm2D(8)
        c2 = paddle.nn.Conv2D(8, 8, 3, padding=1)
        b2 = paddle.nn.BatchNorm2D(8)
        h = paddle.nn.functional.relu(b1(c1(x)))
        h = paddle.nn.functional.relu(b2(c2(h)) + x)       # bn -> add(residual) -> relu
        logits = paddle.nn.functional.adaptive_avg_pool2d(h, 1).reshape([-1, 8])
        loss = paddle.nn.functional.cross_entropy(logits, y)
        paddle.optimizer.SGD(0.1).minimize(loss)
    return main, startup, loss


def test_fused_bn_add_act_pass_training_matches_unfused():
    """fused_bn_add_act_pass: batch_norm -> relu and batch_norm -> add -> relu of a recorded training
    program become one node each; three SGD steps equal the unfused program."""
    paddle.enable_static()
    try:
        rng = np.random.RandomState(0)
        batches = [(rng.randn(4, 8, 6, 6).astype('float32'), rng.randint(0, 8, (4,)).astype('int64'))
                   for _ in range(3)]
        res = []
        for fused in (False, True):
            main, startup, loss = _bn_block_program()
            exe = paddle.static.Executor()
            exe.run(startup)
            if fused:
                nodes, stats = IP.apply_passes(main, passes=['fused_bn_add_act_pass'])
                assert stats.get('fused_bn_add_act_pass') == 2, stats
                main._ir_passes = ['fused_bn_add_act_pass']
                IP._MODE[0] = '1'
            try:
                ls = [float(exe.run(main, feed={'x': xb, 'y': yb}, fetch_list=[loss])[0]) for xb, yb in batches]
            finally:
                IP._MODE[0] = 'auto'
            res.append((ls, [p.numpy().copy() for p in main.all_parameters()]))
        np.testing.assert_allclose(res[0][0], res[1][0], rtol=1e-5, atol=1e-6)
        for a, b in zip(res[0][1], res[1][1]):
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    finally:
        paddle.disable_static()


def test_round6_general_passes_rms_silu_transpose_scale_identity():
    """rms_norm_fuse / silu_fuse / remove_redundant_transpose / matmul_scale_fuse /
    identity_op_clean on a recorded inference program: each rewrites its pattern and the program
    computes the same values."""
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data('x', [4, 16], 'float32')
            h = paddle.nn.RMSNorm(16)(x)                            # composite RMSNorm
            h = h * paddle.nn.functional.sigmoid(h)                 # silu
            h = paddle.transpose(paddle.transpose(h, [1, 0]), [1, 0])  # cancels
            lin = paddle.nn.Linear(16, 8)
            h = lin(h) * 0.5                                        # scale folded into W, b
            h = paddle.cast(h, 'float32') * 1.0 + 0.0               # identities
            out = h.sum(axis=-1)
        exe = paddle.static.Executor()
        xv = np.random.RandomState(1).randn(4, 16).astype('float32')
        ref = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
        passes = ['identity_op_clean_pass', 'remove_redundant_transpose_pass', 'matmul_scale_fuse_pass',
                  'rms_norm_fuse_pass', 'silu_fuse_pass']
        nodes, stats = IP.apply_passes(main, passes=passes, fetch=(main._val[id(out._t)],))
        for p in passes:
            assert stats.get(p, 0) >= 1, (p, stats)
        main._ir_passes = passes
        IP._MODE[0] = '1'
        try:
            got = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
        finally:
            IP._MODE[0] = 'auto'
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    finally:
        paddle.disable_static()
