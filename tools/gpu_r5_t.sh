#!/bin/bash
# round 5 (t): woq decode kernel time split (kernel vs finish), M = 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5t/prof -o woq --output-format csv -- python3 tools/woq_prof.py > gpurun_out/r5t/run.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/r5t/run.log; exit 1; }
python3 tools/ktrace_group.py gpurun_out/r5t/prof woq
