#!/bin/bash
# round 5 (aa): current ERNIE fp8 / bf16 static step profiles
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5aa
for m in fp8 bf16; do
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5aa/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > gpurun_out/r5aa/prof_$m.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5aa/prof_$m.log; exit 1; }
trace=$(find gpurun_out/r5aa/prof_$m -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > gpurun_out/r5aa/ernie_${m}_steady.txt 2>&1
head -50 gpurun_out/r5aa/ernie_${m}_steady.txt | cut -c1-160
rm -f "$trace"
done
timeout -k 10 300 python tools/fp8_cast_bench.py > gpurun_out/r5aa/cast.log 2>&1 || { echo "cast bench failed"; tail -20 gpurun_out/r5aa/cast.log; exit 1; }
grep -v amdgpu gpurun_out/r5aa/cast.log
