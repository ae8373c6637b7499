#!/bin/bash
# round 5 (dd): Llama-2 13B layer-stack steady profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5dd
STEP_MARKER=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5dd/prof -o run --output-format csv -- python3 tools/llama_step.py 3 2 > gpurun_out/r5dd/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5dd/prof.log; exit 1; }
grep llama gpurun_out/r5dd/prof.log
trace=$(find gpurun_out/r5dd/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > gpurun_out/r5dd/llama_steady.txt 2>&1
head -56 gpurun_out/r5dd/llama_steady.txt | cut -c1-170
rm -f "$trace"
