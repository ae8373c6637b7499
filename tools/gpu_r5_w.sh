#!/bin/bash
# round 5 (w): inference fc activation in the GEMM epilogue — numerics, ERNIE predictor latency + census
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_matmul.py tests/test_ir_passes.py > gpurun_out/r5w/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5w/tests.log; exit 1; }
tail -2 gpurun_out/r5w/tests.log
timeout -k 10 300 python tools/ernie_predictor.py > gpurun_out/r5w/pred_ir.log 2>&1 || { echo "pred ir failed"; tail -30 gpurun_out/r5w/pred_ir.log; exit 1; }
grep -v amdgpu gpurun_out/r5w/pred_ir.log | tail -5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5w/prof_ir -o run --output-format csv -- python3 tools/ernie_predictor.py --runs 5 --no-ref > gpurun_out/r5w/prof_ir.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5w/prof_ir.log; exit 1; }
f=$(find gpurun_out/r5w/prof_ir -name '*kernel_stats.csv' | head -1); head -25 "$f" | cut -d, -f1-4 | cut -c1-180
