#!/bin/bash
# One GPU session: kernel numerics tests, smoke, short bench. Each GPU step bounded; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_hip_kernels.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench1.log; exit 1; }
tail -2 gpurun_out/bench1.log
