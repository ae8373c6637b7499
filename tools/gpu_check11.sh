#!/bin/bash
# fused dropout/norm/bias-grad kernels: numerics, full gpu suite, bench, profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "colsum or bias_act_fused or dropout_add_norm or fused_block" --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { echo "fused tests failed"; tail -60 gpurun_out/pytest_fused.log; exit 1; }
tail -1 gpurun_out/pytest_fused.log
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench11.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench11.log; exit 1; }
tail -1 gpurun_out/bench11.log
bash tools/gpu_prof.sh
echo done
