#!/bin/bash
# flash-attention extension kernels: GPU numerics + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_flash_ex.py -x -v --timeout 120 --timeout-method thread > gpurun_out/flash_ex_tests.log 2>&1
rc=$?
tail -5 gpurun_out/flash_ex_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_ex_bench.py > gpurun_out/attn_ex_bench.log 2>&1
rc=$?
cat gpurun_out/attn_ex_bench.log | tail -30
exit $rc
