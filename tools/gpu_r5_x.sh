#!/bin/bash
# round 5 (x): bytecode translation (jit/sot.py) on the GPU — SOT tests + a quick jit/static regression
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5x
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_jit_sot.py > gpurun_out/r5x/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5x/tests.log; exit 1; }
tail -3 gpurun_out/r5x/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jit_sot.py tests/test_ir_passes.py > gpurun_out/r5x/tests2.log 2>&1 || { echo "tests2 failed"; tail -60 gpurun_out/r5x/tests2.log; exit 1; }
tail -2 gpurun_out/r5x/tests2.log
