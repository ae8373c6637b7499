#!/bin/bash
# epilogue-cost diagnostic (stagger sweep), gemm/norm/GPT GPU tests, GPT bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "norm or gpt or dropout or gelu" > gpurun_out/t_a.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_a.log; exit 1; }
tail -2 gpurun_out/t_a.log
timeout -k 10 300 python tools/gemm_epi_cost.py > gpurun_out/epi_cost.log 2>&1 || { echo "epi cost failed"; tail -20 gpurun_out/epi_cost.log; exit 1; }
grep epi gpurun_out/epi_cost.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/bench_a.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_a.log; exit 1; }
tail -1 gpurun_out/bench_a.log | cut -c1-200
