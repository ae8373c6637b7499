#!/bin/bash
# round 5 (v): woq sweep (column tiles x K-split target) after the int4 byte-permute dequant
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v
WOQ_SWEEP=1 timeout -k 10 600 python -u tools/woq_bench.py > gpurun_out/r5v/sweep.log 2>&1 || { echo "sweep failed"; tail -30 gpurun_out/r5v/sweep.log; exit 1; }
grep "best" gpurun_out/r5v/sweep.log
