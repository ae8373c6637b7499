#!/bin/bash
# round 2: 8-phase GEMM correctness (all layouts, ragged, split-K) then speed vs variant 3 + hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "gemm_layouts" --timeout 120 --timeout-method thread > gpurun_out/r2_gemm_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r2_gemm_test.log; exit 1; }
tail -2 gpurun_out/r2_gemm_test.log
GEMM_VARIANTS=9,11,13 timeout -k 10 300 python -u tools/hip_gemm_bench.py > gpurun_out/r2_gemm_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r2_gemm_bench.log; exit 1; }
cat gpurun_out/r2_gemm_bench.log
