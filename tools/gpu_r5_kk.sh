#!/bin/bash
# round 5 (kk): static Linear / FFN / fp8 weight gradients into flat slots: tests, diag, ERNIE steps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5kk
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_hip_ffn_gelu.py tests/test_hip_ir_passes.py tests/test_hip_amp.py tests/test_fp8.py tests/test_static.py tests/test_hip_matmul.py tests/test_models.py > gpurun_out/r5kk/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5kk/tests.log | tail -40; exit 1; }
tail -1 gpurun_out/r5kk/tests.log
timeout -k 10 300 python tools/ernie_slot_diag.py > gpurun_out/r5kk/diag.log 2>&1 || { echo "diag failed"; tail -20 gpurun_out/r5kk/diag.log; exit 1; }
grep -v amdgpu gpurun_out/r5kk/diag.log | tail -2
for m in bf16 fp8; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5kk/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5kk/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5kk/ernie_$m.log | tail -1
done
