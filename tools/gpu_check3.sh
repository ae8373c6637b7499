#!/bin/bash
# stage-3 regression first on the tiny model, then the 1.3B benches and a kernel profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model gpt-tiny --steps 3 --warmup 2 --sharding p_g_os --micro-batch 4 --seq 256 > gpurun_out/bench_tiny.log 2>&1 || { echo "tiny failed"; tail -40 gpurun_out/bench_tiny.log; exit 1; }
tail -1 gpurun_out/bench_tiny.log
for mode in p_g_os dp os_g; do
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --sharding $mode > gpurun_out/bench_$mode.log 2>&1 || { echo "bench $mode failed"; tail -40 gpurun_out/bench_$mode.log; exit 1; }
  tail -1 gpurun_out/bench_$mode.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof3_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof3_bench.log; exit 1; }
echo done
