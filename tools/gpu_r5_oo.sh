#!/bin/bash
# round 5 (oo): GEMM autotune (plain matmuls: hand-written kernel vs library per shape) — tests + matmul bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5oo
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_hip_matmul.py tests/test_jit_sot.py tests/test_hip_ir_passes.py > gpurun_out/r5oo/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5oo/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5oo/tests.log
timeout -k 10 300 python tools/matmul_bench.py > gpurun_out/r5oo/matmul.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r5oo/matmul.log; exit 1; }
grep -v amdgpu gpurun_out/r5oo/matmul.log
for m in bf16; do
PADDLE_AMD_GEMM_AUTOTUNE=1 timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5oo/ernie_tune_$m.log 2>&1 || { echo "ernie failed"; tail -20 gpurun_out/r5oo/ernie_tune_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5oo/ernie_tune_$m.log | tail -1
PADDLE_AMD_GEMM_AUTOTUNE=0 timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5oo/ernie_notune_$m.log 2>&1 || { echo "ernie failed"; tail -20 gpurun_out/r5oo/ernie_notune_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5oo/ernie_notune_$m.log | tail -1
done
