#!/bin/bash
# round 5 (uu): uneven split-K (shorter last slice) — GEMM tests, wgrad split sweep, ERNIE steps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5uu
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_hip_matmul.py tests/test_fp8.py tests/test_hip_ffn_gelu.py > gpurun_out/r5uu/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5uu/tests.log | tail -40; exit 1; }
tail -1 gpurun_out/r5uu/tests.log
timeout -k 10 300 python tools/wgrad_splitk_ab.py > gpurun_out/r5uu/ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r5uu/ab.log; exit 1; }
grep -v amdgpu gpurun_out/r5uu/ab.log | cut -c1-260
for m in bf16 fp8; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5uu/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5uu/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5uu/ernie_$m.log | tail -1
done
