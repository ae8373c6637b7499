#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu13.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu13.log; exit 1; }
tail -1 gpurun_out/pytest_gpu13.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench13.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench13.log; exit 1; }
tail -1 gpurun_out/bench13.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --micro-batch 32 > gpurun_out/bench13_mb32.log 2>&1 || { echo "bench mb32 failed"; tail -40 gpurun_out/bench13_mb32.log; exit 1; }
tail -1 gpurun_out/bench13_mb32.log
bash tools/gpu_prof.sh
python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 5 24
echo done
