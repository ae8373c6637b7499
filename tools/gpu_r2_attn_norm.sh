#!/bin/bash
# flash-attention + fused norm GPU tests, extended attention bench, GPT-3 1.3B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_flash_ex.py -q -m gpu -k "flash or attn or norm or fused or gpt or dropout" --timeout 200 --timeout-method thread > gpurun_out/an_tests.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/an_tests.log | tail -40; exit 1; }
tail -1 gpurun_out/an_tests.log
timeout -k 10 300 python -u tools/attn_ex_bench.py > gpurun_out/attn_ex.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn_ex.log; exit 1; }
grep -v amdgpu gpurun_out/attn_ex.log | head -12
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/gpt_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/gpt_bench.log; exit 1; }
tail -1 gpurun_out/gpt_bench.log
