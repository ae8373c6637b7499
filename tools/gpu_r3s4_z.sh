#!/bin/bash
# session-4 final check at HEAD: smoke, all GPU tests, the 1-GPU bench (GPT-3 1.3B + ResNet50)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s4z_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r3s4z_smoke.log; exit 1; }
tail -1 gpurun_out/r3s4z_smoke.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s4z_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s4z_gputest.log; exit 1; }
tail -2 gpurun_out/r3s4z_gputest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s4z_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r3s4z_bench.log; exit 1; }
tail -1 gpurun_out/r3s4z_bench.log
