#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "decode or kv_cache" --timeout 120 --timeout-method thread > gpurun_out/r2_decode_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r2_decode_test.log; exit 1; }
tail -2 gpurun_out/r2_decode_test.log
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/r2_decode_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r2_decode_bench.log; exit 1; }
cat gpurun_out/r2_decode_bench.log
