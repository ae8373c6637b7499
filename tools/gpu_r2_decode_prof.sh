#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_dec
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec -o run --output-format csv -- python3 tools/decode_bench.py > gpurun_out/prof_dec.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_dec.log; exit 1; }
f=$(find gpurun_out/prof_dec -name "*kernel_stats.csv" | head -1)
head -8 "$f" | cut -c1-220
t=$(find gpurun_out/prof_dec -name "*kernel_trace.csv" | head -1)
rm -f "$t"
