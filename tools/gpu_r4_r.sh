#!/bin/bash
# round 4 (r): woq automatic column-tile / split plan: tests + bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_matmul.py -m gpu -x -q -k "weight_only" --timeout 120 --timeout-method thread > gpurun_out/r4r_woq_tests.log 2>&1 || { echo "woq tests failed"; tail -40 gpurun_out/r4r_woq_tests.log; exit 1; }
tail -2 gpurun_out/r4r_woq_tests.log
timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4r_woq_bench.log 2>&1 || { echo "woq bench failed"; tail -30 gpurun_out/r4r_woq_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4r_woq_bench.log
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/r4r_decode_bench.log 2>&1 || { echo "decode bench failed"; tail -30 gpurun_out/r4r_decode_bench.log; exit 0; }
grep -v amdgpu.ids gpurun_out/r4r_decode_bench.log | tail -12
