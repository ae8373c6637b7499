"""Measures forward / backward times of common paddle ops on the current device and writes the
cost-model table paddlepaddle-paddle_amd/cost_model/static_op_benchmark.json (record keys of the
reference's python/paddle/cost_model/static_op_benchmark.json; times in milliseconds).

usage: python tools/op_benchmark.py [out.json]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddle  # noqa: E402
import paddle.nn.functional as F  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n
    import time
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e3


def case(op, make, f, dtype):
    xs = make(dtype)
    for x in xs:
        if isinstance(x, paddle.Tensor) and x.dtype in (paddle.float32, paddle.bfloat16, paddle.float16):
            x.stop_gradient = False
    with paddle.no_grad():
        tf = timed(lambda: f(*xs))
    out = f(*xs)
    g = paddle.ones_like(out)
    tfb = timed(lambda: f(*xs).backward(g)) if not out.stop_gradient else tf
    cfg = ''.join(f"x{i} (Variable) - dtype: {dtype}, shape: {list(x.shape)}\n" for i, x in enumerate(xs)
                  if isinstance(x, paddle.Tensor))
    return {'name': f'{op}_0', 'op': op, 'op_count': 1, 'config': cfg, 'timestamp': 'mi355x',
            'paddle_gpu_time': f'{tf:.6f}', 'paddle_gpu_time_backward': f'{max(tfb - tf, 0.0):.6f}'}


def R(*shape):
    return lambda dt: [paddle.randn(list(shape)).astype(dt)]


def R2(s1, s2):
    return lambda dt: [paddle.randn(list(s1)).astype(dt), paddle.randn(list(s2)).astype(dt)]


CASES = [
    ('abs', R(16, 128, 257, 257), paddle.abs),
    ('relu', R(16, 128, 257, 257), F.relu),
    ('gelu', R(16, 1024, 8192), F.gelu),
    ('silu', R(16, 1024, 8192), F.silu),
    ('exp', R(16, 1024, 4096), paddle.exp),
    ('add', R2((16, 1024, 2048), (16, 1024, 2048)), paddle.add),
    ('multiply', R2((16, 1024, 2048), (16, 1024, 2048)), paddle.multiply),
    ('matmul', R2((16384, 2048), (2048, 8192)), paddle.matmul),
    ('matmul', R2((4096, 4096), (4096, 4096)), paddle.matmul),
    ('softmax', R(16, 16, 1024, 1024), lambda x: F.softmax(x, -1)),
    ('layer_norm', R(16384, 2048), lambda x: F.layer_norm(x, [2048])),
    ('rms_norm', R(16384, 4096), lambda x: paddle.incubate.nn.functional.fused_rms_norm(
        x, paddle.ones([4096]).astype(x.dtype), None, 1e-6, 1)[0]),
    ('reduce_sum', R(16384, 4096), lambda x: x.sum(-1)),
    ('reduce_mean', R(16384, 4096), lambda x: x.mean(-1)),
    ('transpose', R(64, 512, 1024), lambda x: x.transpose([0, 2, 1])),
    ('concat', R2((64, 512, 1024), (64, 512, 1024)), lambda a, b: paddle.concat([a, b], 1)),
    ('dropout', R(16, 1024, 2048), lambda x: F.dropout(x, 0.1)),
    ('conv2d', R(64, 64, 56, 56), lambda x: F.conv2d(x, paddle.randn([64, 64, 3, 3]).astype(x.dtype), padding=1)),
    ('batch_norm', R(64, 256, 56, 56), lambda x: F.batch_norm(x, paddle.zeros([256]), paddle.ones([256]),
                                                              training=True)),
    ('pool2d', R(64, 64, 112, 112), lambda x: F.max_pool2d(x, 3, 2, 1)),
    ('scaled_dot_product_attention', lambda dt: [paddle.randn([16, 1024, 16, 128]).astype(dt) for _ in range(3)],
     lambda q, k, v: F.scaled_dot_product_attention(q, k, v, is_causal=True)),
]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'paddlepaddle-paddle_amd', 'cost_model',
        'static_op_benchmark.json')
    if torch.cuda.is_available():
        paddle.set_device('gpu')
    recs = []
    for op, make, f in CASES:
        for dt in ('float32', 'bfloat16'):
            if op == 'scaled_dot_product_attention' and dt == 'float32':
                continue
            try:
                recs.append(case(op, make, f, dt))
                print(f"{op:30s} {dt:9s} fwd {recs[-1]['paddle_gpu_time']} ms  bwd {recs[-1]['paddle_gpu_time_backward']} ms",
                      flush=True)
            except Exception as e:  # keep going: the table lists what ran
                print(f"{op} {dt}: {type(e).__name__}: {e}", flush=True)
    with open(out, 'w') as f:
        json.dump(recs, f, indent=1)
    print('wrote', out, len(recs), 'records')


if __name__ == '__main__':
    main()
