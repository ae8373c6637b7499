#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench8.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench8.log; exit 1; }
tail -1 gpurun_out/bench8.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --sharding dp > gpurun_out/bench8_dp.log 2>&1 || { echo "bench dp failed"; tail -40 gpurun_out/bench8_dp.log; exit 1; }
tail -1 gpurun_out/bench8_dp.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof8_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof8_bench.log; exit 1; }
timeout -k 10 600 python bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/bench8_resnet.log 2>&1 || { echo "resnet failed"; tail -40 gpurun_out/bench8_resnet.log; exit 1; }
tail -1 gpurun_out/bench8_resnet.log
echo done
