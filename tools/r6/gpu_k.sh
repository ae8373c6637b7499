#!/bin/bash
# round 6 (k): kernel-level times of the two LayerNorm backward kernels (rocprofv3 stats over tools/norm_bwd_ab.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/norm_bwd_ab.py > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
grep -i "norm_bwd\|colsum" "$f" | cut -c1-220
find $O/prof -name "*kernel_trace.csv" -delete
