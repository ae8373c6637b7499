#!/bin/bash
# int8 KV-cache decode: GPU numerics vs fp32 reference, then bf16-vs-int8 cache timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "decode or kv_cache" --timeout 120 --timeout-method thread > gpurun_out/r3s3_q8_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3_q8_tests.log; exit 1; }
tail -2 gpurun_out/r3s3_q8_tests.log
timeout -k 10 200 python -u tools/decode_q8_bench.py > gpurun_out/r3s3_decode_q8.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r3s3_decode_q8.log; exit 1; }
cat gpurun_out/r3s3_decode_q8.log
