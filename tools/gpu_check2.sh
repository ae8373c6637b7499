#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_hip_kernels.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for mode in p_g_os dp os_g; do
  timeout -k 10 600 python bench.py --steps 6 --warmup 3 --sharding $mode > gpurun_out/bench_$mode.log 2>&1 || { echo "bench $mode failed"; tail -40 gpurun_out/bench_$mode.log; exit 1; }
  tail -1 gpurun_out/bench_$mode.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof2_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof2_bench.log; exit 1; }
echo done
