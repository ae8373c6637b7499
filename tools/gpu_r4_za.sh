#!/bin/bash
# round 4 (za): channel-padded batch norm (ShuffleNetV2 widths) + conv routing tests + zoo scan
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_conv_routing.py tests/test_hip_kernels.py -k "batchnorm or bn or conv" > gpurun_out/r4za_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r4za_tests.log; exit 1; }
tail -5 gpurun_out/r4za_tests.log
timeout -k 10 600 python -u tools/zoo_miopen_scan.py > gpurun_out/r4za_zoo_scan.log 2>&1 || { echo "scan failed"; tail -30 gpurun_out/r4za_zoo_scan.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4za_zoo_scan.log
