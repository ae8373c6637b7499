#!/bin/bash
# round 5 (jj): where the ERNIE static step's parameter-sized add_ come from
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5jj
timeout -k 10 300 python tools/ernie_op_census.py bf16 > gpurun_out/r5jj/census.log 2>&1 || { echo "census failed"; tail -20 gpurun_out/r5jj/census.log; exit 1; }
grep -A40 -- "--- stacks" gpurun_out/r5jj/census.log | cut -c1-600
