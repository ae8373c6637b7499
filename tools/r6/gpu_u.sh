#!/bin/bash
# round 6 (u): column-sum kernels (bias gradients) in round-robin row order: numerics + ERNIE / GPT A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_hip_ffn_gelu.py tests/test_fp8.py -k "bias or act or colsum or gelu or ffn or fp8 or linear" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/cs_order_ab.py > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
grep -v amdgpu $O/ab.log
