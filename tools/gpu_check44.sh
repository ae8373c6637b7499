#!/bin/bash
# stale packed-filter fix: regression test, conv tests, ResNet bench (loss must train)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "conv or fp8" --timeout 120 --timeout-method thread > gpurun_out/pytest44.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest44.log; exit 1; }
tail -1 gpurun_out/pytest44.log
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench44_rn.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/bench44_rn.log; exit 1; }
grep "warmup step" gpurun_out/bench44_rn.log | tail -5
tail -1 gpurun_out/bench44_rn.log
