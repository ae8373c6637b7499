#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu16.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_gpu16.log; exit 1; }
tail -1 gpurun_out/pytest_gpu16.log
timeout -k 10 600 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench16_rn.log 2>&1 || { echo "rn bench failed"; tail -40 gpurun_out/bench16_rn.log; exit 1; }
tail -1 gpurun_out/bench16_rn.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench16.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench16.log; exit 1; }
tail -1 gpurun_out/bench16.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_rn
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 6 > gpurun_out/prof_rn.log 2>&1 || { echo "rn prof failed"; tail -30 gpurun_out/prof_rn.log; exit 1; }
echo done
