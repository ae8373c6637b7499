#!/bin/bash
# round 5 (a): ADVICE-fix GPU tests, then rocprof summaries of the ERNIE fp8 vs bf16 static steps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_matmul.py -k "addmm or woq or weight_only" tests/test_hip_flash_ds.py > gpurun_out/r5a/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
for m in bf16 fp8; do
  timeout -k 10 300 python tools/ernie_step.py $m 5 3 > gpurun_out/r5a/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5a/ernie_$m.log; exit 1; }
  tail -1 gpurun_out/r5a/ernie_$m.log
  STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > gpurun_out/r5a/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 gpurun_out/r5a/prof_$m.log; exit 1; }
  trace=$(find gpurun_out/r5a/prof_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_steady.py "$trace" spin_kernel 3 45 > gpurun_out/r5a/ernie_${m}_steady.txt 2>&1
  head -60 gpurun_out/r5a/ernie_${m}_steady.txt
  rm -f "$trace"
done
