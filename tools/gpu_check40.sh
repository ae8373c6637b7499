#!/bin/bash
# GEMM 5-slot ring variant: numerics + A/B on the GPT shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest40.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest40.log; exit 1; }
tail -1 gpurun_out/pytest40.log
GEMM_VARIANTS=1,3 timeout -k 10 400 python -u tools/hip_gemm_bench.py > gpurun_out/hip_gemm40.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/hip_gemm40.log; exit 1; }
grep -v "splitk=2\|splitk=4" gpurun_out/hip_gemm40.log
