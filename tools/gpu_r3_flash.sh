#!/bin/bash
# flash-attention GPU tests + the plain/ext attention bench (GPT-3 1.3B shapes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_flash_ex.py tests/test_hip_kernels.py -m gpu -k "flash or attn" > gpurun_out/flash_tests.log 2>&1
rc=$?
tail -3 gpurun_out/flash_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_ex_bench.py > gpurun_out/attn_ex_bench.log 2>&1
rc=$?
cat gpurun_out/attn_ex_bench.log | grep -v amdgpu.ids
exit $rc
