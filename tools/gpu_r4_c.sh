#!/bin/bash
# round 4 (c): smoke, full GPU test suite, bench (GPT + ResNet + llama2_13b + ernie_fp8 extra keys)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r4c_smoke.log; exit 1; }
tail -1 gpurun_out/r4c_smoke.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4c_gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/r4c_gputest.log; exit 1; }
tail -3 gpurun_out/r4c_gputest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r4c_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r4c_bench.log; exit 1; }
tail -1 gpurun_out/r4c_bench.log
