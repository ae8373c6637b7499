#!/bin/bash
# round 6 (ac): ERNIE fp8 steady profile on the final tree (bias gradients from the dY cast)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ac; mkdir -p $O
STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/ernie_step.py fp8 3 3 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
trace=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > $O/ernie_fp8_steady.txt 2>&1
head -30 $O/ernie_fp8_steady.txt | cut -c1-150
rm -f "$trace"
