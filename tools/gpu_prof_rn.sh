#!/bin/bash
# steady-state rocprofv3 kernel trace of the ResNet50 bench (5 steps, last 3 aggregated)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_rn_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_rn_bench.log; exit 1; }
tail -1 gpurun_out/prof_rn_bench.log | cut -c1-200
trace=$(find gpurun_out/prof_rn -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" momentum_kernel 3 45 > gpurun_out/prof_rn_steady.txt && head -60 gpurun_out/prof_rn_steady.txt
rm -f "$trace"
