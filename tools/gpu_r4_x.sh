#!/bin/bash
# round 4 (x): stem Cout % 16, MobileNetV2 zero-library step, conv tests, stem / ResNet bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_conv_routing.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r4x_conv_tests.log 2>&1
rc=$?
tail -12 gpurun_out/r4x_conv_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/conv_r4_bench.py > gpurun_out/r4x_conv_bench.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/r4x_conv_bench.log; exit 1; }
grep -i "resnet\|stem" gpurun_out/r4x_conv_bench.log
exit $rc
