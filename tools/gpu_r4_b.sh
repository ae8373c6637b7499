#!/bin/bash
# round 4 (b): matmul / fp8 / woq tests + benches, rccl world-1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
true
true
true
true
timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4b_woq_bench.log 2>&1 || { echo "woq bench failed"; tail -30 gpurun_out/r4b_woq_bench.log; exit 1; }
cat gpurun_out/r4b_woq_bench.log
timeout -k 10 300 python -u tools/matmul_bench.py > gpurun_out/r4b_matmul_bench.log 2>&1 || { echo "matmul bench failed"; tail -30 gpurun_out/r4b_matmul_bench.log; exit 1; }
cat gpurun_out/r4b_matmul_bench.log
timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r4b_fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/r4b_fp8_bench.log; exit 1; }
cat gpurun_out/r4b_fp8_bench.log
