#!/bin/bash
# round 5 (gg): fused GELU FFN (fuse_gemm_epilogue_pass) tests + ERNIE static step bf16 / fp8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5gg
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_hip_ffn_gelu.py tests/test_hip_ir_passes.py tests/test_hip_kernels.py tests/test_static.py > gpurun_out/r5gg/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" gpurun_out/r5gg/tests.log | tail -40; exit 1; }
tail -3 gpurun_out/r5gg/tests.log
for m in bf16 fp8; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > gpurun_out/r5gg/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 gpurun_out/r5gg/ernie_$m.log; exit 1; }
grep -v amdgpu gpurun_out/r5gg/ernie_$m.log | tail -1
done
m=${PROF_MODE:-bf16}
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5gg/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > gpurun_out/r5gg/prof_$m.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5gg/prof_$m.log; exit 1; }
trace=$(find gpurun_out/r5gg/prof_$m -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > gpurun_out/r5gg/ernie_${m}_steady.txt 2>&1
head -30 gpurun_out/r5gg/ernie_${m}_steady.txt | cut -c1-160
rm -f "$trace"
