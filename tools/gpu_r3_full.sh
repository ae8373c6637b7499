#!/bin/bash
# all GPU tests, the 1-GPU bench (GPT-3 1.3B + ResNet50), the MI355X op-benchmark table, and a
# steady-state rocprofv3 profile of the GPT step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3_gputest.log; exit 1; }
tail -2 gpurun_out/r3_gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r3_bench.log; exit 1; }
tail -1 gpurun_out/r3_bench.log
timeout -k 10 300 python -u tools/op_benchmark.py gpurun_out/static_op_benchmark.json > gpurun_out/r3_op_benchmark.log 2>&1 || { echo "op benchmark failed"; tail -20 gpurun_out/r3_op_benchmark.log; exit 1; }
tail -3 gpurun_out/r3_op_benchmark.log
if [ "${PROF:-1}" = "1" ]; then
bash tools/gpu_prof_gpt.sh
fi
