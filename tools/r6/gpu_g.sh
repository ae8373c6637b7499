#!/bin/bash
# round 6 (g): fp8 cast kernel modes (back-to-back timing) + ERNIE fp8 steady profile with the persistent cast
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 200 python -u tools/fp8_cast_bench.py > $O/cast_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/cast_bench.log; exit 1; }
grep -v amdgpu $O/cast_bench.log
m=fp8
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > $O/prof_$m.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_$m.log; exit 1; }
trace=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > $O/ernie_${m}_steady.txt 2>&1
head -20 $O/ernie_${m}_steady.txt | cut -c1-150
grep -i cast_transpose $O/ernie_${m}_steady.txt | cut -c1-150
rm -f "$trace"
