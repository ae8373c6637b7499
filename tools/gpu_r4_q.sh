#!/bin/bash
# round 4 (q): woq default CT 4 + CT 2 variant: tests, sweep, decode layer bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_matmul.py -m gpu -x -q -k "weight_only" --timeout 120 --timeout-method thread > gpurun_out/r4q_woq_tests.log 2>&1 || { echo "woq tests failed"; tail -40 gpurun_out/r4q_woq_tests.log; exit 1; }
tail -2 gpurun_out/r4q_woq_tests.log
WOQ_SWEEP=1 timeout -k 10 600 python -u tools/woq_bench.py > gpurun_out/r4q_woq_sweep.log 2>&1 || { echo "woq sweep failed"; tail -30 gpurun_out/r4q_woq_sweep.log; exit 1; }
grep best gpurun_out/r4q_woq_sweep.log
timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4q_woq_bench.log 2>&1 || { echo "woq bench failed"; tail -30 gpurun_out/r4q_woq_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4q_woq_bench.log
