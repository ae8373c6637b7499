#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "sharding" > gpurun_out/r3s3_t_r.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3_t_r.log; exit 1; }
tail -2 gpurun_out/r3s3_t_r.log
bash tools/gpu_rehearse_2rank.sh
