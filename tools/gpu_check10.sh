#!/bin/bash
# flash bwd variant-1 default: bench + GEMM shape table + rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench_tuned.log 2>&1 || { echo "gemm bench failed"; tail -30 gpurun_out/gemm_bench_tuned.log; exit 1; }
cat gpurun_out/gemm_bench_tuned.log
PADDLE_AMD_GEMM_TUNING=0 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench_untuned.log 2>&1 || { echo "gemm bench failed"; tail -30 gpurun_out/gemm_bench_untuned.log; exit 1; }
cat gpurun_out/gemm_bench_untuned.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench10.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench10.log; exit 1; }
tail -1 gpurun_out/bench10.log
bash tools/gpu_prof.sh
echo done
