#!/bin/bash
# conv kernels: GPU numerics + ResNet50-shape bench vs MIOpen
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "conv" > gpurun_out/conv_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench_d.log 2>&1
