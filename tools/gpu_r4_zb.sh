#!/bin/bash
# round 4 (zb): C_out-padded conv route (SqueezeNet head) + conv routing tests + zoo scan
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_conv_routing.py > gpurun_out/r4zb_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r4zb_tests.log; exit 1; }
tail -3 gpurun_out/r4zb_tests.log
timeout -k 10 600 python -u tools/zoo_miopen_scan.py > gpurun_out/r4zb_zoo_scan.log 2>&1 || { echo "scan failed"; tail -30 gpurun_out/r4zb_zoo_scan.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4zb_zoo_scan.log
