"""Bytecode-level translation (paddle.jit.sot, reference python/paddle/jit/sot/): graph breaks fall
back to Python, captured graphs are recorded into static Programs and run by the Executor, guards
re-translate on new shapes, gradients flow through the captured Programs."""
import numpy as np
import pytest
import torch

import paddle
import paddle.nn.functional as F
from paddle.jit import sot


class _Net(paddle.nn.Layer):
    def __init__(self, d=16, h=32):
        super().__init__()
        self.l1 = paddle.nn.Linear(d, h)
        self.ln = paddle.nn.LayerNorm(h)
        self.l2 = paddle.nn.Linear(h, d)

    def forward(self, x):
        return self.l2(F.gelu(self.ln(self.l1(x)))) + x


def _close(a, b, tol=1e-5):
    np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=tol, atol=tol)


def test_graph_break_on_data_dependent_branch():
    def f(x, y):
        z = F.relu(paddle.matmul(x, y)) + 1
        if float(z.mean()) > 1.0:  # tensor value -> Python: a graph break
            z = z * 2
        else:
            z = z - 1
        return z.sum(axis=-1)
    before = sot.stats()
    tf = sot.symbolic_translate(f)
    paddle.seed(1)
    x, y = paddle.randn([4, 8]), paddle.randn([8, 4])
    _close(tf(x, y), f(x, y))
    _close(tf(x, y), f(x, y))
    st = sot.stats()
    assert st['graphs'] - before['graphs'] >= 2            # split at the break
    assert st['recorded'] - before['recorded'] >= 2        # both sides became Programs
    assert st['calls'] - before['calls'] >= 4              # and served the calls


def test_side_effects_stay_python(capsys):
    calls = []

    def f(x):
        y = x * 3
        calls.append(1)
        print("inside")
        return paddle.tanh(y)
    tf = sot.symbolic_translate(f)
    x = paddle.randn([3, 5])
    _close(tf(x), f(x))
    assert len(calls) == 2 and "inside" in capsys.readouterr().out


def test_guards_retranslate_on_new_shape():
    def f(x):
        return (x * x).sum(axis=0)
    tf = sot.symbolic_translate(f)
    for n in (3, 5, 3):
        x = paddle.randn([n, 4])
        _close(tf(x), f(x))


def test_layer_to_static_sot_forward_and_grads():
    paddle.seed(2)
    net = _Net()
    x = paddle.randn([6, 16])
    ref = _Net.forward(net, x)
    ref.sum().backward()
    g_ref = [p.grad.numpy().copy() for p in net.parameters()]
    net.clear_gradients()
    snet = paddle.jit.to_static(net, backend='sot')
    out = snet(x)
    _close(out, ref)
    out.sum().backward()
    for p, g in zip(net.parameters(), g_ref):
        np.testing.assert_allclose(p.grad.numpy(), g, rtol=1e-5, atol=1e-5)


def test_training_loop_matches_eager():
    def run(translate):
        paddle.seed(3)
        net = _Net()
        opt = paddle.optimizer.AdamW(learning_rate=1e-2, parameters=net.parameters())
        fwd = sot.symbolic_translate(net.forward) if translate else net.forward
        losses = []
        for i in range(3):
            x = paddle.to_tensor(np.random.RandomState(i).randn(8, 16).astype('float32'))
            loss = (fwd(x) ** 2).mean()
            loss.backward()
            opt.step()
            opt.clear_grad()
            losses.append(float(loss))
        return losses
    np.testing.assert_allclose(run(True), run(False), rtol=1e-5)


@pytest.mark.gpu
def test_sot_gpu_bf16_runs_on_executor_kernels(monkeypatch):
    """On the GPU the captured graphs run through the Executor with the GEMMs on the hand-written
    kernels (ops.matmul substitutions) — checked by a spy — and match eager bf16."""
    from paddle.ops import matmul as hm
    paddle.seed(4)
    net = _Net(64, 256)
    net.to(device='gpu', dtype='bfloat16')
    x = paddle.to_tensor(torch.randn(512, 64, device='cuda').bfloat16())
    with paddle.no_grad():
        ref = _Net.forward(net, x)
        hits = []
        subs = hm.static_substitutions()
        from paddle.static import executor as E
        wrapped = {k: (lambda f: (lambda *a, **k: (hits.append(1), f(*a, **k))[1]))(v) for k, v in subs.items()}
        monkeypatch.setattr(E, '_GEMM_SUBS', wrapped)
        out = sot.symbolic_translate(net.forward)(x)
    torch.cuda.synchronize()
    err = (out._t.float() - ref._t.float()).abs().max().item() / ref._t.float().abs().max().item()
    assert err < 2e-2, err
    assert hits, "captured GEMMs did not run on the Executor's kernel substitutions"


# ------------------------------------------------------------ the framework's own opcode translator
from paddle.jit.opcode_translator import OpcodeTranslator, stats as ot_stats  # noqa: E402

_SCALE = 2.0


def _scaled(x):
    return x * _SCALE


class _Block(paddle.nn.Layer):
    def __init__(self, d):
        super().__init__()
        self.fc = paddle.nn.Linear(d, d)
        self.use_act = True

    def forward(self, x):
        y = self.fc(x)
        if self.use_act:  # a Python attribute: baked, guarded
            y = F.relu(y)
        return y


class _Stack(paddle.nn.Layer):
    def __init__(self, d=8, n=3):
        super().__init__()
        self.blocks = paddle.nn.LayerList([_Block(d) for _ in range(n)])
        self.drop = paddle.nn.Dropout(0.5)

    def forward(self, x, extra=None):
        outs = []
        for b in self.blocks:              # unrolled: one region for the whole stack
            x = b(x)
            outs.append(x.mean())
        h = {'y': self.drop(x), 'means': [o * 1 for o in outs]}
        if extra is not None:
            h['y'] = h['y'] + extra
        return h


def test_opcode_translator_one_region_unrolled_and_replayed():
    paddle.seed(5)
    net = _Stack()
    net.eval()
    tr = OpcodeTranslator(net.forward)
    x = paddle.randn([4, 8])
    before = ot_stats()
    out = tr(x)
    mid = ot_stats()
    out2 = tr(x)
    after = ot_stats()
    ref = net(x)
    _close(out['y'], ref['y'])
    _close(out2['y'], ref['y'])
    assert len(out['means']) == 3
    assert mid['regions'] - before['regions'] == 1 and mid['breaks'] == before['breaks']  # no graph break
    assert after['regions'] == mid['regions'] and after['hits'] - mid['hits'] == 1        # replayed, not retraced
    out3 = tr(x, extra=paddle.ones([4, 8]))                                               # new kwargs state
    _close(out3['y'], ref['y'] + 1)


def test_opcode_translator_guards_attribute_global_and_training_flag():
    global _SCALE
    paddle.seed(6)
    net = _Stack()
    net.eval()
    tr = OpcodeTranslator(net.forward)
    x = paddle.randn([4, 8])
    _close(tr(x)['y'], net(x)['y'])
    net.blocks[1].use_act = False       # attribute the translation branched on
    _close(tr(x)['y'], net(x)['y'])
    net.train()                         # dropout on: a different region (training flags guarded)
    paddle.seed(9)
    y1 = tr(x)['y']
    assert float((y1 == 0).astype('float32').mean()) > 0.2
    net.eval()
    tg = OpcodeTranslator(_scaled)
    _close(tg(x), x * 2.0)
    _SCALE = 3.0                        # global the translation read
    try:
        _close(tg(x), x * 3.0)
    finally:
        _SCALE = 2.0


def test_opcode_translator_breaks_side_effects_and_eager_fallbacks():
    log = []

    def helper(t):
        log.append(float(t.sum()))      # tensor value + outer list: runs concretely
        return t * 2

    def f(x):
        y = paddle.exp(x)
        z = helper(y)
        s = f"{z.shape[0]} rows"        # Python string from a shape: fine inside a region
        return z + 1, s

    def gen(x):                         # generator: not modelled, runs eagerly
        yield x * 2
    tr = OpcodeTranslator(f)
    x = paddle.randn([3, 4])
    for _ in range(2):
        out, s = tr(x)
        _close(out, paddle.exp(x) * 2 + 1)
        assert s == '3 rows'
    assert len(log) == 2
    tg = OpcodeTranslator(lambda t: list(gen(t))[0])
    _close(tg(x), x * 2)


def test_opcode_translator_input_gradients_and_closures():
    w = paddle.randn([4, 4])

    def f(x, k=2):
        sq = [x * i for i in range(k)]          # list comprehension (inlined function)
        g = lambda t: paddle.matmul(t, w)       # closure over a captured tensor
        return g(sum(sq[1:], sq[0])).sum()
    tr = OpcodeTranslator(f)
    x = paddle.randn([3, 4])
    x.stop_gradient = False
    loss = tr(x, k=3)
    loss.backward()
    ref_x = x.detach()
    ref_x.stop_gradient = False
    (paddle.matmul(ref_x * 3, w)).sum().backward()
    _close(x.grad, ref_x.grad)


@pytest.mark.parametrize("family", ['gpt', 'llama', 'ernie'])
def test_opcode_translator_model_zoo_single_region(family):
    """GPT / Llama / ERNIE forwards translate as ONE region each (no graph break: function-level
    imports, comprehensions, the models' own helpers inlined), equal eager, and train (gradients
    on every parameter); two translations in a row do not share recorded tensors (the RoPE tables
    of a recording belong to its program)."""
    from paddle.models import gpt, llama, ernie
    paddle.seed(7)
    rng = np.random.RandomState(7)
    if family == 'gpt':
        net = gpt.GPTForPretraining(gpt.gpt_config('gpt-tiny'))
    elif family == 'llama':
        net = llama.LlamaForCausalLM(llama.llama_config('llama-tiny'))
    else:
        net = ernie.ErnieForSequenceClassification(ernie.ernie_config('ernie-tiny'))
    ids = paddle.to_tensor(rng.randint(0, 512, (2, 16)))
    net.eval()
    ref = net(ids)
    ref = ref if isinstance(ref, paddle.Tensor) else ref[0]
    for _ in range(2):
        tr = OpcodeTranslator(net.forward)
        before = ot_stats()
        out = tr(ids)
        out = out if isinstance(out, paddle.Tensor) else out[0]
        after = ot_stats()
        assert after['regions'] - before['regions'] == 1 and after['breaks'] == before['breaks']
        _close(out, ref, 1e-5)
    net.train()
    out = tr(ids)
    (out if isinstance(out, paddle.Tensor) else out[0]).mean().backward()
    assert all(p.grad is not None for p in net.parameters())


@pytest.mark.gpu
def test_sot_gpt_tiny_gpu_bf16_forward_and_train():
    """GPT-tiny in bf16 on the GPU through the opcode translator: one region replayed by the
    Executor (GEMM substitutions, IR fusion passes) equals eager within bf16 tolerance, and a
    training call produces gradients for every parameter."""
    from paddle.models import gpt
    paddle.set_device('gpu')
    try:
        paddle.seed(8)
        net = gpt.GPTForPretraining(gpt.gpt_config('gpt-tiny'))
        net.to(dtype='bfloat16')
        ids = paddle.to_tensor(np.random.RandomState(8).randint(0, 512, (4, 64)))
        net.eval()
        with paddle.no_grad():
            ref = net(ids)
            tr = OpcodeTranslator(net.forward)
            out = tr(ids)
            out = tr(ids)
        ref = ref if isinstance(ref, paddle.Tensor) else ref[0]
        out = out if isinstance(out, paddle.Tensor) else out[0]
        r, o = ref._t.float(), out._t.float()
        assert float((o - r).abs().max() / r.abs().max()) < 3e-2
        net.train()
        y = tr(ids)
        (y if isinstance(y, paddle.Tensor) else y[0]).astype('float32').mean().backward()
        assert all(p.grad is not None for p in net.parameters())
    finally:
        paddle.set_device('cpu')


def test_opcode_translator_with_blocks_pass_through_and_cache():
    """`with` blocks are entered / exited concretely around translated regions (grad mode and AMP
    state guard the regions), objects the caller passed in are handed back (not copies), per-call
    lists and context managers do not defeat the region cache, and an exception inside a block
    closes it."""
    paddle.seed(10)
    lin = paddle.nn.Linear(4, 4)

    def f(x, acc):
        with paddle.no_grad():
            y = lin(x) * 2
        z = lin(x) + y
        acc.append(float(z.sum()))   # break: the caller's own list
        out = []
        for i in range(2):
            out.append(z * i)
        return out, acc

    tr = OpcodeTranslator(f)
    x = paddle.randn([3, 4])
    acc = []
    before = None
    for it in range(3):
        out, a2 = tr(x, acc)
        assert a2 is acc and len(acc) == it + 1
        assert paddle.is_grad_enabled()
        ref = lin(x) + lin(x).detach() * 2
        _close(out[1], ref)
        assert out[1].stop_gradient is False and out[0].stop_gradient is False
        if it == 0:
            before = ot_stats()['regions']
    assert ot_stats()['regions'] == before  # calls 2 and 3 replayed every region

    def g(x):
        with paddle.no_grad():
            y = x * 2
            raise ValueError('boom')
        return y
    tg = OpcodeTranslator(g)
    with pytest.raises(ValueError):
        tg(x)
    assert paddle.is_grad_enabled()


def test_opcode_translator_region_created_iterators_and_closures_replay():
    """A region that creates an iterator (a for loop over range / a list) and breaks inside the
    loop hands the iterator on by source and position, so every replay iterates afresh (it used
    to bake the recording's exhausted iterator: the second call skipped the loop); a closure
    created over the region's values is never baked into a template."""
    import numpy as np
    from paddle.jit import sot

    def loop_setitem(x):
        z = paddle.zeros_like(x)
        for i in range(x.shape[0]):
            z[i] = x[i] * i
        return z

    def loop_list(x):
        acc = x * 0
        for w in [1.0, 2.0, 3.0]:
            acc[0] = acc[0] + x[0] * w
        return acc

    def closure(x):
        c = 0

        def inc():
            nonlocal c
            c += 1
            return x * c
        inc()
        return inc()

    def loop_break_append(x):  # a bound list.append left on the stack at a mutation break
        r = []
        for i in range(3):
            if x.sum() > 1e9:
                break
            r.append(x + i)
        return paddle.concat(r)

    x = paddle.randn([4, 3])
    for fn in (loop_setitem, loop_list, closure, loop_break_append):
        st = sot.symbolic_translate(fn)
        ref = fn(x).numpy()
        for _ in range(3):
            np.testing.assert_allclose(st(x).numpy(), ref, rtol=1e-6, atol=1e-6)
        x2 = paddle.randn([4, 3])
        np.testing.assert_allclose(st(x2).numpy(), fn(x2).numpy(), rtol=1e-6, atol=1e-6)


def test_opcode_translator_wrapped_functions_bind_their_own_parameters():
    """A functools.wraps wrapper (paddle.no_grad() as a decorator: ``def w(*a, **k)``) is bound by
    its own code object's parameters, not by the wrapped function's signature."""
    import numpy as np
    from paddle.jit import sot

    @paddle.no_grad()
    def f(x, scale=2.0):
        return x * scale

    def g(x):
        return f(x) + f(x, scale=3.0)

    x = paddle.randn([3, 4])
    for fn in (f, g):
        st = sot.symbolic_translate(fn)
        for _ in range(2):
            np.testing.assert_allclose(st(x).numpy(), fn(x).numpy(), rtol=1e-6)


def test_opcode_translator_translates_layer_instances():
    """symbolic_translate(layer) runs the Layer's __call__ (hooks, then forward) through the
    translator — recorded regions, no eager fallback — and matches the eager Layer, including a
    training-mode dropout under the same seed and a train / eval switch."""
    import numpy as np
    from paddle.jit import sot

    class Blk(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.l1, self.l2 = paddle.nn.Linear(8, 16), paddle.nn.Linear(16, 8)
            self.drop = paddle.nn.Dropout(0.3)

        def forward(self, x, scale=1.0):
            h = paddle.nn.functional.gelu(self.l1(x))
            if self.training:
                h = self.drop(h)
            return self.l2(h) * scale

    m = Blk()
    st = sot.symbolic_translate(m)
    before = sot.stats()
    x = paddle.randn([4, 8])
    for mode in ('train', 'eval', 'train'):
        getattr(m, mode)()
        for _ in range(2):
            paddle.seed(3)
            got = st(x, scale=2.0)
            paddle.seed(3)
            np.testing.assert_allclose(got.numpy(), m(x, scale=2.0).numpy(), rtol=1e-5, atol=1e-6)
    after = sot.stats()
    assert after['eager_calls'] == before['eager_calls']
    assert after['recorded'] > before['recorded']
