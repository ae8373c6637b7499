#!/bin/bash
# Records the flagship bench's GEMM shapes, then tunes them one by one (TunableOp) into
# paddlepaddle-paddle_amd/configs/gemm_tuning_gfx950.csv (copied back under gpurun_out/configs/).
set -o pipefail
mkdir -p gpurun_out/configs
OUT=paddlepaddle-paddle_amd/configs/gemm_tuning_gfx950.csv
rm -f $OUT gpurun_out/untuned.csv
PADDLE_AMD_GEMM_TUNING=0 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 \
PYTORCH_TUNABLEOP_UNTUNED_FILENAME=gpurun_out/untuned.csv \
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 > gpurun_out/record_gemms.log 2>&1 || { echo "record failed"; tail -20 gpurun_out/record_gemms.log; exit 1; }
ls gpurun_out/
UNT=$(ls gpurun_out/untuned*.csv | head -1)
wc -l $UNT
timeout -k 10 1000 python tools/tune_gemms.py $UNT $OUT || { echo "tune failed"; exit 1; }
ls -la paddlepaddle-paddle_amd/configs/; cp $OUT* gpurun_out/configs/
