#!/bin/bash
# round 4 (b): matmul / fp8 / woq tests + benches, rccl world-1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_hip_matmul.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1 || { echo "matmul tests failed"; tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -2 gpurun_out/r4b_tests.log
timeout -k 10 300 python -u -m pytest tests/test_rccl_world1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b_rccl.log 2>&1 || { echo "rccl tests failed"; tail -40 gpurun_out/r4b_rccl.log; exit 1; }
tail -2 gpurun_out/r4b_rccl.log
timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4b_woq_bench.log 2>&1 || { echo "woq bench failed"; tail -30 gpurun_out/r4b_woq_bench.log; exit 1; }
cat gpurun_out/r4b_woq_bench.log
timeout -k 10 300 python -u tools/matmul_bench.py > gpurun_out/r4b_matmul_bench.log 2>&1 || { echo "matmul bench failed"; tail -30 gpurun_out/r4b_matmul_bench.log; exit 1; }
cat gpurun_out/r4b_matmul_bench.log
timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r4b_fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/r4b_fp8_bench.log; exit 1; }
cat gpurun_out/r4b_fp8_bench.log
