#!/bin/bash
# round 5 (h): software-pipelined flash forward at D = 64 — numerics tests, then the A/B bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_hip_flash_sp.py > gpurun_out/r5h/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5h/tests.log; exit 1; }
tail -2 gpurun_out/r5h/tests.log
timeout -k 10 300 python tools/attn_sp_ab.py > gpurun_out/r5h/ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r5h/ab.log; exit 1; }
cat gpurun_out/r5h/ab.log | grep -v amdgpu.ids
