#!/bin/bash
# round 4 (l): graph-timed woq plan sweep (K-split target blocks x register stages)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
WOQ_SWEEP=1 timeout -k 10 600 python -u tools/woq_bench.py > gpurun_out/r4l_woq_sweep.log 2>&1 || { echo "woq sweep failed"; tail -30 gpurun_out/r4l_woq_sweep.log; exit 1; }
grep best gpurun_out/r4l_woq_sweep.log
