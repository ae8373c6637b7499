#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 "$@" > gpurun_out/prof_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*kernel_stats.csv" | head
