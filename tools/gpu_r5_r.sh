#!/bin/bash
# round 5 (r): deep-filter stem (AlexNet 11x11/4), C_in % 8 padding (ShuffleNet) — routing tests, zoo scan
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5r
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_conv_routing.py -k "stem or cin" > gpurun_out/r5r/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5r/tests.log; exit 1; }
tail -3 gpurun_out/r5r/tests.log
timeout -k 10 400 python -u tools/zoo_miopen_scan.py alexnet shufflenet_v2_x1_0 > gpurun_out/r5r/zoo.log 2>&1 || { echo "zoo failed"; tail -30 gpurun_out/r5r/zoo.log; exit 1; }
grep -v Warning gpurun_out/r5r/zoo.log | tail -4
