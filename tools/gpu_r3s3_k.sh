#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "skinny" > gpurun_out/r3s3_t_k.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3_t_k.log; exit 1; }
tail -2 gpurun_out/r3s3_t_k.log
timeout -k 10 300 python tools/decode_gemm_bench.py > gpurun_out/r3s3_decode_gemm.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3s3_decode_gemm.log; exit 1; }
grep -v amdgpu gpurun_out/r3s3_decode_gemm.log
