#!/bin/bash
# round 6 (p): GPT-3 1.3B steady profile after the AdamW change (one vector per lane, temporal accesses)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gpt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-resnet --no-extra > $O/prof_gpt_bench.log 2>&1 || { echo "gpt prof failed"; tail -30 $O/prof_gpt_bench.log; exit 1; }
trace=$(find $O/prof_gpt -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" adamw_kernel 3 60 > $O/gpt_steady.txt && head -30 $O/gpt_steady.txt | cut -c1-160
grep -i "adamw\|sumsq" $O/gpt_steady.txt | cut -c1-160
rm -f "$trace"
