#!/bin/bash
# round 5 (q): int8 FMT per-Linear device time (hipGraph replay)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5q
timeout -k 10 300 python -u tools/fmt_int8_bench.py > gpurun_out/r5q/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5q/bench.log; exit 1; }
cat gpurun_out/r5q/bench.log
