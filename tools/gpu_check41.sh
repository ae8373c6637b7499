#!/bin/bash
# hand-written conv2d: numerics, per-shape A/B vs MIOpen, ResNet bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "conv" --timeout 120 --timeout-method thread > gpurun_out/pytest41.log 2>&1 || { echo "conv tests failed"; tail -40 gpurun_out/pytest41.log; exit 1; }
tail -1 gpurun_out/pytest41.log
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv41.log 2>&1 || { echo "conv bench failed"; tail -20 gpurun_out/conv41.log; exit 1; }
cat gpurun_out/conv41.log
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench41_rn.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/bench41_rn.log; exit 1; }
tail -1 gpurun_out/bench41_rn.log
