#!/bin/bash
# hand-written MFMA GEMM: numerics, then per-shape A/B vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest24.log 2>&1 || { echo "gemm tests failed"; tail -40 gpurun_out/pytest24.log; exit 1; }
tail -1 gpurun_out/pytest24.log
timeout -k 10 300 python -u tools/hip_gemm_bench.py > gpurun_out/hip_gemm24.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/hip_gemm24.log; exit 1; }
cat gpurun_out/hip_gemm24.log
timeout -k 10 200 python -u tools/hip_gemm_bench.py square > gpurun_out/hip_gemm24_sq.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/hip_gemm24_sq.log; exit 1; }
cat gpurun_out/hip_gemm24_sq.log
