#!/bin/bash
# round 5 (b): fusion-pass GPU tests, ERNIE static step bf16 / fp8 with the IR passes, profiles
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hip_ir_passes.py > gpurun_out/r5b/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5b/tests.log; exit 1; }
tail -3 gpurun_out/r5b/tests.log
for m in bf16 fp8; do
  timeout -k 10 300 python tools/ernie_step.py $m 5 3 > gpurun_out/r5b/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -30 gpurun_out/r5b/ernie_$m.log; exit 1; }
  tail -1 gpurun_out/r5b/ernie_$m.log
done
for m in bf16 fp8; do
  STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > gpurun_out/r5b/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 gpurun_out/r5b/prof_$m.log; exit 1; }
  trace=$(find gpurun_out/r5b/prof_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > gpurun_out/r5b/ernie_${m}_steady.txt 2>&1
  head -30 gpurun_out/r5b/ernie_${m}_steady.txt
  rm -f "$trace"
done
