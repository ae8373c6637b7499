#!/bin/bash
# Measures the fastest hipBLASLt/rocBLAS solution for every GEMM shape of the flagship
# benchmark (TunableOp) and writes paddlepaddle-paddle_amd/configs/gemm_tuning_gfx950.csv.
set -o pipefail
mkdir -p gpurun_out
OUT=paddlepaddle-paddle_amd/configs/gemm_tuning_gfx950.csv
rm -f $OUT
PADDLE_AMD_GEMM_TUNING=0 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_VERBOSE=1 \
  timeout -k 10 900 python bench.py --steps 1 --warmup 1 > gpurun_out/tune_gemms.log 2>&1 || { echo "tuning failed"; tail -30 gpurun_out/tune_gemms.log; exit 1; }
mkdir -p gpurun_out/configs && cp $OUT gpurun_out/configs/
wc -l $OUT
