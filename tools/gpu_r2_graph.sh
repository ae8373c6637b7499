#!/bin/bash
# training-step hipGraph: GPU test, then ResNet50 bench eager vs --graph (same box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -q -m gpu -k "graph" --timeout 200 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/graph_tests.log | tail -40; exit 1; }
tail -1 gpurun_out/graph_tests.log
timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn_eager.log 2>&1 || { echo "eager bench failed"; tail -20 gpurun_out/rn_eager.log; exit 1; }
tail -1 gpurun_out/rn_eager.log | cut -c1-160
timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 --graph > gpurun_out/rn_graph.log 2>&1 || { echo "graph bench failed"; tail -30 gpurun_out/rn_graph.log; exit 1; }
tail -1 gpurun_out/rn_graph.log | cut -c1-400
