#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "colsum or bias_act_fused or dropout_add_norm or fused_block" --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { echo "fused tests failed"; tail -60 gpurun_out/pytest_fused.log; exit 1; }
tail -1 gpurun_out/pytest_fused.log
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench12.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench12.log; exit 1; }
tail -1 gpurun_out/bench12.log
bash tools/gpu_prof.sh
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench_split.log 2>&1 || { echo "gemm bench failed"; tail -30 gpurun_out/gemm_bench_split.log; exit 1; }
grep -E "split|wgrad" gpurun_out/gemm_bench_split.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_rn
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2 > gpurun_out/prof_rn.log 2>&1 || { echo "rn prof failed"; tail -30 gpurun_out/prof_rn.log; exit 1; }
tail -1 gpurun_out/prof_rn.log
echo done
