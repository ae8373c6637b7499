#!/bin/bash
# HIP weight-gradient GEMM in the GPT step: tests, then A/B of the flagship bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "gemm or gpt" --timeout 120 --timeout-method thread > gpurun_out/pytest21.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest21.log; exit 1; }
tail -1 gpurun_out/pytest21.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench21_hip.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench21_hip.log; exit 1; }
tail -1 gpurun_out/bench21_hip.log
PADDLE_AMD_HIP_GEMM=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench21_lib.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench21_lib.log; exit 1; }
tail -1 gpurun_out/bench21_lib.log
