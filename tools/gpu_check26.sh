#!/bin/bash
# full GPU test tier + both benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest26.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|error" gpurun_out/pytest26.log | head -30; tail -30 gpurun_out/pytest26.log; exit 1; }
tail -1 gpurun_out/pytest26.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench26.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench26.log; exit 1; }
tail -1 gpurun_out/bench26.log
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench26_rn.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/bench26_rn.log; exit 1; }
tail -1 gpurun_out/bench26_rn.log
