#!/bin/bash
# fused BN statistics (conv / GEMM epilogue): new tests, full GPU suite, bench, ResNet A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "bn_stats or epi5 or from_parts or batchnorm or resnet or im2col" > gpurun_out/r3s3_t_bn.log 2>&1 || { echo "bn tests failed"; tail -40 gpurun_out/r3s3_t_bn.log; exit 1; }
tail -2 gpurun_out/r3s3_t_bn.log
for v in 0 1; do
  PADDLE_AMD_CONV_BN_STATS=$v timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3s3_rn_$v.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/r3s3_rn_$v.log; exit 1; }
  echo "BN_STATS=$v $(tail -1 gpurun_out/r3s3_rn_$v.log)"
done
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s3_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s3_gputest.log; exit 1; }
tail -2 gpurun_out/r3s3_gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s3_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r3s3_bench.log; exit 1; }
tail -1 gpurun_out/r3s3_bench.log
