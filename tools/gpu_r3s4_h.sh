#!/bin/bash
# wide transpose kernel: transpose tests, all GPU tests, bench, steady GPT profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt
timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -x -q -k transpose2d --timeout 120 --timeout-method thread > gpurun_out/r3s4h_tr.log 2>&1 || { echo "transpose tests failed"; tail -30 gpurun_out/r3s4h_tr.log; exit 1; }
tail -1 gpurun_out/r3s4h_tr.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s4h_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s4h_gputest.log; exit 1; }
tail -2 gpurun_out/r3s4h_gputest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s4h_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r3s4h_bench.log; exit 1; }
tail -1 gpurun_out/r3s4h_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-resnet > gpurun_out/prof_gpt_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_gpt_bench.log; exit 1; }
trace=$(find gpurun_out/prof_gpt -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" adamw_kernel 3 40 > gpurun_out/r3s4h_gpt_steady.txt && head -30 gpurun_out/r3s4h_gpt_steady.txt
rm -f "$trace"
