#!/bin/bash
# conv numerics, ResNet50 bench (hand-written conv backward) and its steady-state kernel profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_rn
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "conv" > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
timeout -k 10 400 python -u bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/rn_bench.log 2>&1 || { tail -30 gpurun_out/rn_bench.log; exit 1; }
tail -1 gpurun_out/rn_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2 > gpurun_out/prof_rn_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_rn_bench.log; exit 1; }
trace=$(find gpurun_out/prof_rn -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" momentum_kernel 3 45 > gpurun_out/prof_rn_steady.txt && head -60 gpurun_out/prof_rn_steady.txt
rm -f "$trace"
