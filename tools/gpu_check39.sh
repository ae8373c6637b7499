#!/bin/bash
# norm backward row pipelining: numerics + GPT bench + kernel stats
set -o pipefail
mkdir -p gpurun_out/prof39
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "norm or dropout or fused or gpt or colsum" --timeout 120 --timeout-method thread > gpurun_out/pytest39.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest39.log; exit 1; }
tail -1 gpurun_out/pytest39.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench39.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench39.log; exit 1; }
tail -1 gpurun_out/bench39.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof39 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof39.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof39.log; exit 1; }
echo profiled
