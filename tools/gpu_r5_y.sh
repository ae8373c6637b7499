#!/bin/bash
# round 5 (y): conv3d_transpose on the 2-D transposed-conv kernels
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5y
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_conv_routing.py -k "conv3d or transpose" > gpurun_out/r5y/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5y/tests.log; exit 1; }
tail -2 gpurun_out/r5y/tests.log
