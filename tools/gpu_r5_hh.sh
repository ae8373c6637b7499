#!/bin/bash
# round 5 (hh): embedding tests, ERNIE steps, torch-op census of the ERNIE bf16 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5hh
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "embedding" > gpurun_out/r5hh/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5hh/tests.log | tail -40; exit 1; }
tail -2 gpurun_out/r5hh/tests.log
for m in bf16 fp8; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5hh/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5hh/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5hh/ernie_$m.log | tail -1
done
timeout -k 10 300 python tools/ernie_op_census.py bf16 > gpurun_out/r5hh/census.log 2>&1 || { echo "census failed"; tail -20 gpurun_out/r5hh/census.log; exit 1; }
grep -v amdgpu gpurun_out/r5hh/census.log | tail -40
