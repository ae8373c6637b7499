#!/bin/bash
# round 5 (ii): embedding tests, ERNIE steps, torch-op census of the ERNIE bf16 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ii
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_hip_ffn_gelu.py tests/test_hip_ir_passes.py tests/test_hip_amp.py tests/test_fp8.py tests/test_static.py tests/test_hip_matmul.py > gpurun_out/r5ii/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5ii/tests.log | tail -40; exit 1; }
tail -2 gpurun_out/r5ii/tests.log
for m in bf16 fp8; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5ii/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5ii/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5ii/ernie_$m.log | tail -1
done
timeout -k 10 300 python tools/ernie_op_census.py bf16 > gpurun_out/r5ii/census.log 2>&1 || { echo "census failed"; tail -20 gpurun_out/r5ii/census.log; exit 1; }
grep -v amdgpu gpurun_out/r5ii/census.log | tail -40
