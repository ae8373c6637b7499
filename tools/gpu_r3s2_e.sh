#!/bin/bash
# staged weight-gradient epilogue: bitwise test, then bench A/B (GPT) of PADDLE_AMD_GEMM_STAGED9
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "staged or wgrad or grouped" > gpurun_out/t_e.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_e.log; exit 1; }
tail -2 gpurun_out/t_e.log
VAR=PADDLE_AMD_GEMM_STAGED9 VALS="0 1" ROUNDS=2 bash tools/gpu_ab_env.sh
