#!/bin/bash
# steady-state rocprofv3 kernel trace of the GPT-3 1.3B bench (5 steps, last 3 aggregated)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-resnet --no-extra > gpurun_out/prof_gpt_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_gpt_bench.log; exit 1; }
tail -1 gpurun_out/prof_gpt_bench.log | cut -c1-200
trace=$(find gpurun_out/prof_gpt -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" adamw_kernel 3 40 > gpurun_out/prof_gpt_steady.txt && head -90 gpurun_out/prof_gpt_steady.txt
python3 -c "import sys" && rm -f "$trace"
