#!/bin/bash
# round 4 (a): matmul family on the hand-written GEMM + 8-phase fp8 GEMM: tests, benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_matmul.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { echo "matmul tests failed"; tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -2 gpurun_out/r4a_tests.log
timeout -k 10 300 python -u tools/matmul_bench.py > gpurun_out/r4a_matmul_bench.log 2>&1 || { echo "matmul bench failed"; tail -30 gpurun_out/r4a_matmul_bench.log; exit 1; }
cat gpurun_out/r4a_matmul_bench.log
timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r4a_fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/r4a_fp8_bench.log; exit 1; }
cat gpurun_out/r4a_fp8_bench.log
timeout -k 10 300 python -u -m pytest tests/test_rccl_world1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_rccl.log 2>&1 || { echo "rccl tests failed"; tail -40 gpurun_out/r4a_rccl.log; exit 1; }
tail -2 gpurun_out/r4a_rccl.log
