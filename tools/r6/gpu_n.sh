#!/bin/bash
# round 6 (n): steady-state kernel profiles of the current tree: ERNIE fp8 + bf16 (static AMP), GPT-3 1.3B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
for m in fp8 bf16; do
  STEP_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python3 tools/ernie_step.py $m 3 3 > $O/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 $O/prof_$m.log; exit 1; }
  trace=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_steady.py "$trace" spin_kernel 3 60 > $O/ernie_${m}_steady.txt 2>&1
  head -45 $O/ernie_${m}_steady.txt | cut -c1-160
  rm -f "$trace"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gpt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-resnet --no-extra > $O/prof_gpt_bench.log 2>&1 || { echo "gpt prof failed"; tail -30 $O/prof_gpt_bench.log; exit 1; }
trace=$(find $O/prof_gpt -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" adamw_kernel 3 60 > $O/gpt_steady.txt && head -50 $O/gpt_steady.txt | cut -c1-160
rm -f "$trace"
