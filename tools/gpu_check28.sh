#!/bin/bash
# ERNIE static AMP-O2 GPU test alone (serialised), then the full GPU tier and both benches
set -o pipefail
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_static.py -x -v -m gpu -k ernie --timeout 120 --timeout-method thread > gpurun_out/pytest28a.log 2>&1 || { echo "ernie failed"; grep -v "^frame\|^  File" gpurun_out/pytest28a.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest28a.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest28.log 2>&1 || { echo "gpu tests failed"; grep -v "^frame\|^  File" gpurun_out/pytest28.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest28.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench28.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench28.log; exit 1; }
tail -1 gpurun_out/bench28.log
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench28_rn.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/bench28_rn.log; exit 1; }
tail -1 gpurun_out/bench28_rn.log
