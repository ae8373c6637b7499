#!/bin/bash
# round 5 (ee): fused QKV -> RoPE -> flash attention (Llama) — tests, llama step before/after
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ee
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_rope_flash.py tests/test_hip_kernels.py -k "rope or llama or flash" > gpurun_out/r5ee/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5ee/tests.log; exit 1; }
tail -1 gpurun_out/r5ee/tests.log
timeout -k 10 600 python tools/llama_step.py 5 2 > gpurun_out/r5ee/llama.log 2>&1 || { echo "llama failed"; tail -30 gpurun_out/r5ee/llama.log; exit 1; }
tail -1 gpurun_out/r5ee/llama.log
