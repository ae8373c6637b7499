#!/bin/bash
# captured training steps under a host LR scheduler (device learning rate refilled per replay)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v -k "graph" --timeout 120 --timeout-method thread > gpurun_out/r3s4b_graph_tests.log 2>&1 || { echo "graph tests failed"; tail -60 gpurun_out/r3s4b_graph_tests.log; exit 1; }
tail -15 gpurun_out/r3s4b_graph_tests.log
