#!/bin/bash
# round 5 (u): woq fused finish — numerics tests, graph-timed bench A/B (fused vs finish kernel)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_matmul.py tests/test_fmt_int8.py tests/test_hip_quant.py > gpurun_out/r5u/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5u/tests.log; exit 1; }
tail -2 gpurun_out/r5u/tests.log
timeout -k 10 600 python -u tools/woq_bench.py > gpurun_out/r5u/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5u/bench.log; exit 1; }
grep -v amdgpu gpurun_out/r5u/bench.log
timeout -k 10 300 python -u tools/fmt_int8_bench.py > gpurun_out/r5u/fmt.log 2>&1 || { echo "fmt bench failed"; tail -30 gpurun_out/r5u/fmt.log; exit 1; }
grep "^{" gpurun_out/r5u/fmt.log | head -8
