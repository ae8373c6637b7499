"""Native auto-growth best-fit allocator (csrc/alloc/allocator.cpp; reference
paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc).  CPU: the block logic on the
host backend (best fit, split, neighbour merge, per-stream pools, idle-chunk release, cap).
GPU: a GPT-tiny training run in a fresh process with the allocator installed matches the
default-allocator run, and the statistics are consistent."""
import json
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def L():
    from paddle.device.cuda import allocator as A
    lib = A.lib()
    assert lib.pa_alloc_live_blocks() == 0
    assert lib.pa_alloc_config(1, 1, 0) == 0  # host backend, 1 MiB chunks
    return A


def _stats(A, dev=7):
    return A.stats(dev)


def test_best_fit_split_merge(L):
    lib, dev = L.lib(), 7
    a = lib.pa_alloc_malloc(1000, dev, None)      # -> 1024 B block from a 1 MiB chunk
    b = lib.pa_alloc_malloc(4096, dev, None)
    c = lib.pa_alloc_malloc(1, dev, None)
    assert a % 512 == 0 and b == a + 1024 and c == b + 4096
    st = _stats(L, dev)
    assert st['allocated'] == 1024 + 4096 + 512 and st['num_chunks'] == 1 and st['reserved'] == 1 << 20
    lib.pa_alloc_free(b)
    d = lib.pa_alloc_malloc(2000, dev, None)      # best fit: the 4 KiB hole, not the chunk tail
    assert d == b
    lib.pa_alloc_free(a)
    lib.pa_alloc_free(d)
    lib.pa_alloc_free(c)                           # everything merges back into one free block
    assert L.largest_free_block(dev) == 1 << 20
    assert _stats(L, dev)['allocated'] == 0
    big = lib.pa_alloc_malloc(3 << 20, dev, None)  # larger than a chunk: an exact-size chunk
    assert _stats(L, dev)['num_chunks'] == 2
    lib.pa_alloc_free(big)
    assert lib.pa_alloc_empty_cache(dev) == (1 << 20) + (3 << 20)
    st = _stats(L, dev)
    assert st['reserved'] == 0 and st['num_chunks'] == 0 and st['peak_reserved'] == 4 << 20


def test_streams_do_not_share_blocks(L):
    lib, dev = L.lib(), 6
    s1, s2 = 0x1000, 0x2000
    a = lib.pa_alloc_malloc(512, dev, s1)
    lib.pa_alloc_free(a)
    b = lib.pa_alloc_malloc(512, dev, s2)          # s1's free block is not handed to s2
    assert _stats(L, dev)['num_chunks'] == 2
    c = lib.pa_alloc_malloc(512, dev, s1)
    assert c == a
    for p in (b, c):
        lib.pa_alloc_free(p)
    lib.pa_alloc_empty_cache(dev)


def test_random_workload_no_overlap(L):
    import ctypes
    lib, dev = L.lib(), 5
    rng = random.Random(0)
    live = {}
    for it in range(3000):
        if live and rng.random() < 0.45:
            p = rng.choice(list(live))
            n, tag = live.pop(p)
            buf = (ctypes.c_ubyte * n).from_address(p)
            assert all(v == tag for v in bytes(buf[:min(n, 64)])), "block contents overwritten"
            lib.pa_alloc_free(p)
        else:
            n = rng.choice([1, 100, 512, 700, 4096, 10000, 65536, 300000])
            p = lib.pa_alloc_malloc(n, dev, None)
            assert p and p % 512 == 0
            for q, (m, _) in live.items():
                assert p + n <= q or q + m <= p, "overlapping blocks"
            tag = it & 0xFF
            ctypes.memset(p, tag, n)
            live[p] = (n, tag)
    for p in list(live):
        lib.pa_alloc_free(p)
    st = _stats(L, dev)
    assert st['allocated'] == 0 and st['num_allocs'] == st['num_frees']
    assert L.largest_free_block(dev) >= 1 << 20   # fully coalesced chunks
    lib.pa_alloc_empty_cache(dev)
    assert _stats(L, dev)['reserved'] == 0


def test_reserved_cap(L):
    lib, dev = L.lib(), 4
    assert lib.pa_alloc_config(1, 1, 2) == 0        # 2 MiB cap
    try:
        a = lib.pa_alloc_malloc(1 << 20, dev, None)
        b = lib.pa_alloc_malloc(1 << 20, dev, None)
        assert a and b
        assert lib.pa_alloc_malloc(1 << 20, dev, None) is None
        assert _stats(L, dev)['num_ooms'] == 1
        lib.pa_alloc_free(a)
        lib.pa_alloc_free(b)
        lib.pa_alloc_empty_cache(dev)
    finally:
        lib.pa_alloc_config(1, 1, 0)


_SCRIPT = r'''
import json, sys
sys.path.insert(0, {root!r})
import paddle
from paddle.models.gpt import gpt_config, GPTForPretraining
paddle.set_device('gpu:0')
paddle.seed(0)
cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
model = GPTForPretraining(cfg)
opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters(), multi_precision=True)
model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
ids = paddle.randint(0, cfg.vocab_size, [4, 129])
losses = []
for _ in range(4):
    loss = model.loss(model(ids[:, :-1]), ids[:, 1:])
    loss.backward(); opt.step(); opt.clear_grad()
    losses.append(float(loss))
from paddle.device import cuda
from paddle.device.cuda import allocator as A
out = {{'losses': losses, 'native': A.is_enabled(), 'allocated': cuda.memory_allocated(),
       'reserved': cuda.memory_reserved(), 'peak': cuda.max_memory_allocated()}}
if A.is_enabled():
    out['stats'] = A.stats(0)
print(json.dumps(out))
'''


@pytest.mark.gpu
def test_native_allocator_trains_like_default():
    outs = []
    for native in ('0', '1'):
        env = dict(os.environ, FLAGS_use_native_allocator=native)
        r = subprocess.run([sys.executable, '-c', _SCRIPT.format(root=ROOT)], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    base, nat = outs
    assert not base['native'] and nat['native']
    for a, b in zip(base['losses'], nat['losses']):
        assert abs(a - b) <= 2e-3 * max(1.0, abs(a)), (base['losses'], nat['losses'])
    st = nat['stats']
    assert 0 < st['allocated'] <= st['reserved'] and st['peak_allocated'] >= st['allocated']
    assert nat['allocated'] == st['allocated'] and st['num_chunks'] >= 1 and st['num_ooms'] == 0
