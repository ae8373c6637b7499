#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || { echo "attn bench failed"; tail -30 gpurun_out/attn_bench.log; exit 1; }
cat gpurun_out/attn_bench.log
PADDLE_AMD_GEMM_TUNING=0 timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_untuned.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_untuned.log; exit 1; }
tail -1 gpurun_out/bench_untuned.log
bash tools/tune_gemms.sh || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_tuned.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log
echo done
