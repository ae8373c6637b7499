#!/bin/bash
# round 6 (e): batched fp8 weight cast — tests, ERNIE fp8 vs bf16, fp8 steady profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_hip_ffn_gelu.py tests/test_fp8.py > gpurun_out/r6e/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r6e/tests.log | tail -40; exit 1; }
tail -1 gpurun_out/r6e/tests.log
for m in fp8 bf16; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r6e/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r6e/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r6e/ernie_$m.log | tail -1
done
m=fp8
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > gpurun_out/r6e/prof_$m.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6e/prof_$m.log; exit 1; }
trace=$(find gpurun_out/r6e/prof_$m -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > gpurun_out/r6e/ernie_${m}_steady.txt 2>&1
head -24 gpurun_out/r6e/ernie_${m}_steady.txt | cut -c1-150
rm -f "$trace"
