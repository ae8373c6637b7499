#!/bin/bash
# full GPU tier + both benches (conv backward policy)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest34.log 2>&1 || { echo "gpu tests failed"; grep -v "^frame\|^  File" gpurun_out/pytest34.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest34.log
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench34_rn.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/bench34_rn.log; exit 1; }
tail -1 gpurun_out/bench34_rn.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench34.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench34.log; exit 1; }
tail -1 gpurun_out/bench34.log
