#!/bin/bash
# round 4 (w): conv forward channel padding (C % 32 != 0): conv tests + ResNet50 bench (no-regression check)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_conv_routing.py tests/test_hip_kernels.py -m gpu -x -q -k "conv or resnet or bn" --timeout 240 --timeout-method thread > gpurun_out/r4w_conv_tests.log 2>&1 || { echo "conv tests failed"; tail -40 gpurun_out/r4w_conv_tests.log; exit 1; }
tail -2 gpurun_out/r4w_conv_tests.log
timeout -k 10 600 python -u tools/conv_r4_bench.py > gpurun_out/r4w_conv_bench.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/r4w_conv_bench.log; exit 1; }
grep -i "resnet\|stem" gpurun_out/r4w_conv_bench.log
