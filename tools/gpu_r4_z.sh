#!/bin/bash
# round 4 (z): vision-zoo scan for library (MIOpen) kernels in a training step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/zoo_miopen_scan.py > gpurun_out/r4z_zoo_scan.log 2>&1 || { echo "scan failed"; tail -30 gpurun_out/r4z_zoo_scan.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4z_zoo_scan.log
