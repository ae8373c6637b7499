#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/blaslt_probe > gpurun_out/blaslt_probe.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/blaslt_probe.log; exit 1; }
cat gpurun_out/blaslt_probe.log
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "adamw or fused or colsum or norm" --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu14.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu14.log; exit 1; }
tail -1 gpurun_out/pytest_gpu14.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench14.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench14.log; exit 1; }
tail -1 gpurun_out/bench14.log
bash tools/gpu_prof.sh
python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 5 16
echo done
