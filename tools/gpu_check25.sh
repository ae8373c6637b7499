#!/bin/bash
# hand-written fp8 GEMM: numerics + fp8 linear, then A/B vs torch._scaled_mm (hipBLASLt fp8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/pytest25.log 2>&1 || { echo "fp8 tests failed"; tail -40 gpurun_out/pytest25.log; exit 1; }
tail -1 gpurun_out/pytest25.log
timeout -k 10 300 python -u tools/hip_gemm_bench.py fp8 > gpurun_out/hip_gemm25_fp8.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/hip_gemm25_fp8.log; exit 1; }
cat gpurun_out/hip_gemm25_fp8.log
