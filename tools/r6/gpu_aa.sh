#!/bin/bash
# round 6 (aa): fp8 Linear / FFN bias gradients from the dY cast's column sums: numerics + ERNIE fp8 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_fp8.py tests/test_hip_ffn_gelu.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/fp8_bias_ab.py > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
grep -v amdgpu $O/ab.log
