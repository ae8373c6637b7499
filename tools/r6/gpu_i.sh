#!/bin/bash
# round 6 (i): fused_bn_add_act GPU test + the full bench on the current tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_ir_passes.py tests/test_jit_sot.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
