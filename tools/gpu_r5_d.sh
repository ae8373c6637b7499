#!/bin/bash
# round 5 (d): fusion + linear-routing tests, ERNIE bf16 / fp8 timing + bf16 profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5d
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_hip_ir_passes.py tests/test_hip_matmul.py > gpurun_out/r5d/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5d/tests.log; exit 1; }
tail -2 gpurun_out/r5d/tests.log
for m in bf16 fp8; do
  timeout -k 10 300 python tools/ernie_step.py $m 5 3 > gpurun_out/r5d/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -30 gpurun_out/r5d/ernie_$m.log; exit 1; }
  tail -1 gpurun_out/r5d/ernie_$m.log
done
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5d/prof_bf16 -o run --output-format csv -- python3 tools/ernie_step.py bf16 3 3 > gpurun_out/r5d/prof_bf16.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5d/prof_bf16.log; exit 1; }
trace=$(find gpurun_out/r5d/prof_bf16 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 30 > gpurun_out/r5d/ernie_bf16_steady.txt 2>&1
head -36 gpurun_out/r5d/ernie_bf16_steady.txt
rm -f "$trace"
