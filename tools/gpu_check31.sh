#!/bin/bash
# flash-attention backward 8-wave variant: numerics (variants 1, 3), A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "flash" --timeout 120 --timeout-method thread > gpurun_out/pytest31.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest31.log; exit 1; }
tail -1 gpurun_out/pytest31.log
FA_VARIANTS=1,3,2 timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn31.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn31.log; exit 1; }
cat gpurun_out/attn31.log
