#!/bin/bash
# round 4 (e): materialised-dS flash backward (tests + attention A/B + GPT bench A/B), conv
# layout debug, remaining conv tests, fp8 / woq / wide-attention benches, RCCL order trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_flash_ds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_flash_ds_tests.log 2>&1 || { echo "ds tests failed"; tail -60 gpurun_out/r4e_flash_ds_tests.log; exit 1; }
tail -3 gpurun_out/r4e_flash_ds_tests.log
FA_DS_AB=1 timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r4e_attn_ds_ab.log 2>&1 || { echo "attn ab failed"; tail -30 gpurun_out/r4e_attn_ds_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4e_attn_ds_ab.log
timeout -k 10 300 python -u tools/resnet_layout_grad_diff.py > gpurun_out/r4e_resnet_grad_diff.log 2>&1 || { echo "grad diff failed"; tail -30 gpurun_out/r4e_resnet_grad_diff.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4e_resnet_grad_diff.log
timeout -k 10 600 python -u -m pytest tests/test_hip_conv_routing.py -q --timeout 120 --timeout-method thread > gpurun_out/r4e_conv_tests.log 2>&1; tail -5 gpurun_out/r4e_conv_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-resnet --no-extra > gpurun_out/r4e_bench_gpt_recompute.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4e_bench_gpt_recompute.log; exit 1; }
tail -1 gpurun_out/r4e_bench_gpt_recompute.log | cut -c1-220
PADDLE_AMD_FA_DS_BWD=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-resnet --no-extra > gpurun_out/r4e_bench_gpt_ds.log 2>&1 || { echo "bench ds failed"; tail -20 gpurun_out/r4e_bench_gpt_ds.log; exit 1; }
tail -1 gpurun_out/r4e_bench_gpt_ds.log | cut -c1-220
