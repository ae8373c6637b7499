#!/bin/bash
# round 4 (d): conv routing / depthwise / stem tests + bench, wide-head-dim flash tests + bench,
# RCCL ordering trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_conv_routing.py -x -q --timeout 120 --timeout-method thread --deselect tests/test_hip_conv_routing.py::test_resnet50_nchw_default_no_miopen > gpurun_out/r4d_conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/r4d_conv_tests.log; exit 1; }
timeout -k 10 300 python -u tools/resnet_layout_grad_diff.py > gpurun_out/r4d_resnet_grad_diff.log 2>&1 || { echo "grad diff failed"; tail -30 gpurun_out/r4d_resnet_grad_diff.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4d_resnet_grad_diff.log
tail -3 gpurun_out/r4d_conv_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hip_flash_wide.py tests/test_hip_flash_ex.py tests/test_fp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_flash_tests.log 2>&1 || { echo "flash tests failed"; tail -60 gpurun_out/r4d_flash_tests.log; exit 1; }
tail -3 gpurun_out/r4d_flash_tests.log
timeout -k 10 600 python -u tools/conv_r4_bench.py > gpurun_out/r4d_conv_bench.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/r4d_conv_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4d_conv_bench.log
timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r4d_fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/r4d_fp8_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4d_fp8_bench.log
FA_SHAPES=wide timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r4d_attn_wide.log 2>&1 || { echo "attn bench failed"; tail -30 gpurun_out/r4d_attn_wide.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4d_attn_wide.log
rm -rf gpurun_out/rccl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rccl -- python3 tools/rccl_order_trace.py > gpurun_out/r4d_rccl_run.log 2>&1 || { echo "rccl trace failed"; tail -30 gpurun_out/r4d_rccl_run.log; exit 1; }
f=$(find gpurun_out/rccl -name '*kernel_trace.csv' | head -1)
python3 tools/rccl_order_trace.py --report "$f" > gpurun_out/r4d_rccl_order.txt 2>&1
head -40 gpurun_out/r4d_rccl_order.txt
WOQ_SWEEP=1 timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4d_woq_sweep.log 2>&1 || { echo "woq sweep failed"; tail -30 gpurun_out/r4d_woq_sweep.log; exit 1; }
grep best gpurun_out/r4d_woq_sweep.log
