#!/bin/bash
# GPU tests (all), GPT-3 1.3B bench, steady-state kernel profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r2_gputest.log; exit 1; }
tail -2 gpurun_out/r2_gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r2_bench.log; exit 1; }
tail -1 gpurun_out/r2_bench.log
if [ "${PROF:-1}" = "1" ]; then
bash tools/gpu_prof_gpt.sh
fi
