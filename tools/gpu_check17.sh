#!/bin/bash
# A/B of the GEMM solution table on ONE box: bench with the committed table, retune longer, bench again
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "batchnorm or momentum" --timeout 120 --timeout-method thread > gpurun_out/pytest17.log 2>&1 || { echo "bn tests failed"; tail -40 gpurun_out/pytest17.log; exit 1; }
tail -1 gpurun_out/pytest17.log
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench17_rn.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/bench17_rn.log; exit 1; }
tail -1 gpurun_out/bench17_rn.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench17_before.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench17_before.log; exit 1; }
tail -1 gpurun_out/bench17_before.log
TUNE_MS=40 TUNE_ITERS=30 bash tools/tune_gemms.sh > gpurun_out/tune17.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune17.log; exit 1; }
tail -3 gpurun_out/tune17.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench17_after.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench17_after.log; exit 1; }
tail -1 gpurun_out/bench17_after.log
echo done
