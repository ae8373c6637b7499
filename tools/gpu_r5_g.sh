#!/bin/bash
# round 5 (g): forced-collective (1-rank RCCL) GPT-3 1.3B stage-3 step: RCCL / compute overlap
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5g
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5g/rccl -o run -- python3 tools/rccl_order_trace.py --gpt13 > gpurun_out/r5g/rccl.log 2>&1 || { echo "trace failed"; tail -30 gpurun_out/r5g/rccl.log; exit 1; }
trace=$(find gpurun_out/r5g/rccl -name "*kernel_trace.csv" | head -1)
python3 tools/rccl_order_trace.py --overlap "$trace" | tee gpurun_out/r5g/overlap.txt
python3 tools/rccl_order_trace.py --report "$trace" > gpurun_out/r5g/order.txt || true
head -25 gpurun_out/r5g/order.txt
cp "$trace" gpurun_out/r5g/trace_keep.csv 2>/dev/null; rm -f "$trace"
