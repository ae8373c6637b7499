#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || { echo "attn bench failed"; tail -30 gpurun_out/attn_bench.log; exit 1; }
cat gpurun_out/attn_bench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_p_g_os.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_p_g_os.log; exit 1; }
tail -1 gpurun_out/bench_p_g_os.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof4_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof4_bench.log; exit 1; }
echo done
