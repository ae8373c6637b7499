#!/bin/bash
# round 5 (ww): uneven split-K for the fp8 weight gradients — tests, split sweep, ERNIE steps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ww
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_fp8.py tests/test_hip_ffn_gelu.py tests/test_hip_amp.py > gpurun_out/r5ww/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5ww/tests.log | tail -40; exit 1; }
tail -1 gpurun_out/r5ww/tests.log
timeout -k 10 300 python tools/fp8_wgrad_splitk_ab.py > gpurun_out/r5ww/ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r5ww/ab.log; exit 1; }
grep -v amdgpu gpurun_out/r5ww/ab.log
for m in fp8 bf16; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5ww/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5ww/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5ww/ernie_$m.log | tail -1
done
