#!/bin/bash
# flash-attention longest-first grid order: numerics + attention bench + GPT bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "flash or gpt" --timeout 120 --timeout-method thread > gpurun_out/pytest35.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest35.log; exit 1; }
tail -1 gpurun_out/pytest35.log
FA_VARIANTS=1,3 timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn35.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn35.log; exit 1; }
cat gpurun_out/attn35.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench35.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench35.log; exit 1; }
tail -1 gpurun_out/bench35.log
