#!/bin/bash
# full GPU test suite, then the 1-GPU bench (headline + ResNet50)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/bench.log
exit $rc
