"""ERNIE-3.0-base sequence classification exported as a reference ProgramDesc (.pdmodel +
.pdiparams) and run by paddle.inference in bf16 on the GPU: IR fusion passes on (default) or off
(--no-ir).  Prints the per-run latency and the max |fused - unfused| of the logits.

usage: python tools/ernie_predictor.py [--no-ir] [--runs N] [--batch B] [--seq S]"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
from paddle import static, inference as I  # noqa: E402
from paddle.models import ernie_config, ErnieForSequenceClassification  # noqa: E402


def export(prefix, S):
    paddle.seed(0)
    paddle.enable_static()
    try:
        cfg = ernie_config('ernie-3.0-base')
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            ids = static.data('ids', [None, S], 'int64')
            model = ErnieForSequenceClassification(cfg, num_classes=2)
            model.eval()
            logits = model(ids)
        static.save_inference_model(prefix, [ids], [logits], static.Executor(paddle.CPUPlace()), program=main)
    finally:
        paddle.disable_static()


def predictor(prefix, ir):
    c = I.Config(prefix + '.pdmodel', prefix + '.pdiparams')
    c.enable_use_gpu(1024, 0, I.PrecisionType.Bfloat16)
    c.switch_ir_optim(ir)
    return I.create_predictor(c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--no-ir', action='store_true')
    ap.add_argument('--runs', type=int, default=10)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--seq', type=int, default=128)
    ap.add_argument('--no-ref', action='store_true', help='skip the unfused reference run (rocprof census)')
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    prefix = os.path.join(d, 'ernie')
    export(prefix, a.seq)
    ids = np.random.RandomState(0).randint(1, 40000, size=(a.batch, a.seq)).astype('int64')
    ids[1, a.seq // 2:] = 0  # padding
    x = paddle.to_tensor(ids, place=paddle.CUDAPlace(0))
    p = predictor(prefix, not a.no_ir)
    assert getattr(p._program, '_pdmodel', False), 'not a ProgramDesc import'
    for _ in range(3):
        out = p.run([x])[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.runs):
        out = p.run([x])[0]
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.runs * 1e3
    from paddle.static import ir_passes as IP
    print(f"ir={'off' if a.no_ir else 'on'} {ms:.3f} ms/run  passes {IP.fusion_stats(p._program)}", flush=True)
    if not a.no_ir and not a.no_ref:
        ref = predictor(prefix, False).run([x])[0].astype('float32').numpy()
        print(f"max |fused - unfused| logits {np.abs(out.astype('float32').numpy() - ref).max():.4g} (|logits| max "
              f"{np.abs(ref).max():.3g})", flush=True)


if __name__ == '__main__':
    main()
