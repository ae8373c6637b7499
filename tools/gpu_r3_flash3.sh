#!/bin/bash
# flash tests on the double-buffered kernels, then the pipe A/B
set -o pipefail
mkdir -p gpurun_out
PA_FA_BWD_VARIANT=4 PA_FA_FWD_PIPE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_flash_ex.py tests/test_hip_kernels.py -m gpu -k "flash or attn" > gpurun_out/flash_tests_pipe.log 2>&1
rc=$?
tail -3 gpurun_out/flash_tests_pipe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_pipe_ab.py > gpurun_out/attn_pipe_ab.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/attn_pipe_ab.log
exit $rc
