#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -x -q -m gpu -k flash > gpurun_out/pytest_flash_v2.log 2>&1 || { echo "flash v2 failed"; tail -40 gpurun_out/pytest_flash_v2.log; exit 1; }
tail -1 gpurun_out/pytest_flash_v2.log
PA_FA_BWD_VARIANT=1 timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -x -q -m gpu -k flash > gpurun_out/pytest_flash_v1.log 2>&1 || { echo "flash v1 failed"; tail -40 gpurun_out/pytest_flash_v1.log; exit 1; }
tail -1 gpurun_out/pytest_flash_v1.log
PA_FA_BWD_VARIANT=1 timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench_v1.log 2>&1 || { echo "attn v1 failed"; tail -30 gpurun_out/attn_bench_v1.log; exit 1; }
PA_FA_BWD_VARIANT=2 timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench_v2.log 2>&1 || { echo "attn v2 failed"; tail -30 gpurun_out/attn_bench_v2.log; exit 1; }
grep causal gpurun_out/attn_bench_v1.log; grep causal gpurun_out/attn_bench_v2.log
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench9.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench9.log; exit 1; }
tail -1 gpurun_out/bench9.log
echo done
