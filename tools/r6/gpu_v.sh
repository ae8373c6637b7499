#!/bin/bash
# round 6 (v): Llama-2 13B layer-stack steady profile on the current tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6v; mkdir -p $O
STEP_MARKER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/llama_step.py 3 2 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
trace=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" spin_kernel 3 40 > $O/llama_steady.txt 2>&1
head -40 $O/llama_steady.txt | cut -c1-170
rm -f "$trace"
