"""Offline GEMM tuning for the flagship bench (TunableOp), one shape at a time with progress.

Each recorded GEMM line (BLAS column-major m, n, k, transA/transB) is replayed as the torch
row-major call that produced it — mm(X, Y) or addmm(bias, X, Y) with Y = op(A), X = op(B) —
with tuning enabled, so TunableOp times every hipBLASLt/rocBLAS solution for that shape and
keeps the fastest.  Winners are written to the DB after every shape.
"""
import os
import sys
import time

import torch

untuned, out = sys.argv[1], sys.argv[2]
lines = []
with open(untuned) as f:
    for ln in f:
        if ln.startswith(("Gemm", "ScaledGemm")) and ln not in lines:
            lines.append(ln.strip())
print(f"{len(lines)} GEMM shapes to tune", flush=True)
t = torch.cuda.tunable
t.enable(True)
t.tuning_enable(True)
t.set_filename(out)
t.set_max_tuning_duration(int(os.environ.get('TUNE_MS', '10')))
t.set_max_tuning_iterations(int(os.environ.get('TUNE_ITERS', '20')))


def _write_partial(path):
    """Progress snapshot (TunableOp itself writes the final table at process exit)."""
    with open(path, 'w') as f:
        for k, v in t.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for r in t.get_results():
            f.write(','.join(str(x) for x in r) + '\n')


dt = {'BFloat16': torch.bfloat16, 'Half': torch.float16, 'float': torch.float32}
dev = torch.device('cuda', 0)
for i, ln in enumerate(lines):
    t0 = time.time()
    op, rest = ln.split(',', 1)
    sig, dtype_name, _ = (op.split('_') + [''])[:3]
    dtype = dt[op.split('_')[1]]
    trans = rest.split('_')[0]
    m, n, k = (int(v) for v in rest.split('_')[1:4])
    ta, tb = trans[0] == 't', trans[1] == 't'
    a = torch.randn((m, k) if ta else (k, m), device=dev, dtype=dtype)
    b = torch.randn((k, n) if tb else (n, k), device=dev, dtype=dtype)
    Y = a.t() if ta else a
    X = b.t() if tb else b
    if sig == 'GemmAndBiasTunableOp':
        torch.addmm(torch.randn(m, device=dev, dtype=dtype), X, Y)
    else:
        torch.mm(X, Y)
    torch.cuda.synchronize()
    _write_partial(out + '.partial')
    print(f"[{i + 1}/{len(lines)}] {ln[:110]}  ({time.time() - t0:.1f}s)", flush=True)
print("tuned; results in", out, flush=True)
