#!/bin/bash
# round 5 (bb): weight-gradient split-K A/B on ERNIE / GPT shapes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5bb
timeout -k 10 300 python tools/wgrad_splitk_ab.py > gpurun_out/r5bb/ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r5bb/ab.log; exit 1; }
grep -v amdgpu gpurun_out/r5bb/ab.log
