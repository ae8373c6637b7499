#!/bin/bash
# round 5 (cc): ERNIE bf16 / fp8 static steps after the one-round split-K rule; GEMM tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5cc
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_matmul.py > gpurun_out/r5cc/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5cc/tests.log; exit 1; }
tail -1 gpurun_out/r5cc/tests.log
for m in bf16 fp8 bf16 fp8; do
  timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5cc/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -30 gpurun_out/r5cc/ernie_$m.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/r5cc/ernie_$m.log)"
done
