#!/bin/bash
# full GPU suite, then bench A/B (GPT + ResNet50) of the staged epilogue: 0 = register stores, 4 = wave-local staged
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s2_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s2_gputest.log; exit 1; }
tail -2 gpurun_out/r3s2_gputest.log
BENCH_ARGS=" " VAR=PADDLE_AMD_GEMM_STAGED VALS="0 4" ROUNDS=2 bash tools/gpu_ab_env.sh
