#!/bin/bash
# round 5 (s): conv regression tests + the whole vision-zoo library scan
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_conv_routing.py tests/test_hip_kernels.py -k "conv or stem or bn" > gpurun_out/r5s/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5s/tests.log; exit 1; }
tail -3 gpurun_out/r5s/tests.log
timeout -k 10 900 python -u tools/zoo_miopen_scan.py > gpurun_out/r5s/zoo.log 2>&1 || { echo "zoo failed"; tail -30 gpurun_out/r5s/zoo.log; exit 1; }
grep -v Warning gpurun_out/r5s/zoo.log | tail -16
