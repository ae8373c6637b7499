"""Offline GEMM tuning for the flagship bench (TunableOp), one shape at a time with progress.

Step 1 (separate process): run bench.py with PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 to list shapes.
Step 2 (this script): tune each recorded GEMM line, writing the winners to the committed DB.
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
            lines.append(ln)
print(f"{len(lines)} GEMM shapes to tune", flush=True)
t = torch.cuda.tunable
t.enable(True)
t.tuning_enable(True)
t.set_filename(out)
t.set_max_tuning_duration(int(os.environ.get('TUNE_MS', '8')))
t.set_max_tuning_iterations(int(os.environ.get('TUNE_ITERS', '20')))
torch.cuda.set_device(0)
for i, ln in enumerate(lines):
    t0 = time.time()
    t._process_single_offline_gemm(ln, 0)
    t.write_file()
    print(f"[{i + 1}/{len(lines)}] {ln.strip()[:120]}  ({time.time() - t0:.1f}s)", flush=True)
print("tuned; results in", out, flush=True)
