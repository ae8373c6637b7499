#!/bin/bash
# AdamW streaming A/B + optimizer numerics
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "adamw or momentum" --timeout 120 --timeout-method thread > gpurun_out/pytest37.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest37.log; exit 1; }
tail -1 gpurun_out/pytest37.log
timeout -k 10 300 python -u tools/adamw_bench.py > gpurun_out/adamw37.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/adamw37.log; exit 1; }
cat gpurun_out/adamw37.log
