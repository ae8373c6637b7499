#!/bin/bash
# round 5 (c): fp8 split-K tests, ERNIE GEMM A/B, ERNIE bf16/fp8 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_hip_matmul.py -k "fp8 or amp or int8" tests/test_fp8.py tests/test_hip_amp.py > gpurun_out/r5c/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5c/tests.log; exit 1; }
tail -2 gpurun_out/r5c/tests.log
timeout -k 10 300 python tools/ernie_gemm_ab.py > gpurun_out/r5c/gemm_ab.log 2>&1 || { echo "gemm ab failed"; tail -30 gpurun_out/r5c/gemm_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5c/gemm_ab.log
for m in bf16 fp8; do
  timeout -k 10 300 python tools/ernie_step.py $m 5 3 > gpurun_out/r5c/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -30 gpurun_out/r5c/ernie_$m.log; exit 1; }
  tail -1 gpurun_out/r5c/ernie_$m.log
done
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5c/prof_fp8 -o run --output-format csv -- python3 tools/ernie_step.py fp8 3 3 > gpurun_out/r5c/prof_fp8.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5c/prof_fp8.log; exit 1; }
trace=$(find gpurun_out/r5c/prof_fp8 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 30 > gpurun_out/r5c/ernie_fp8_steady.txt 2>&1
head -36 gpurun_out/r5c/ernie_fp8_steady.txt
rm -f "$trace"
timeout -k 10 300 python tools/matmul_bench.py > gpurun_out/r5c/matmul_bench.log 2>&1 || { echo "matmul bench failed"; tail -20 gpurun_out/r5c/matmul_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5c/matmul_bench.log
