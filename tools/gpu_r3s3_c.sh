#!/bin/bash
# ResNet50 steady-state profiles: epilogue BN statistics on / off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0; do
  mkdir -p gpurun_out/prof_rn$v
  PADDLE_AMD_CONV_BN_STATS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn$v -o run --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2 > gpurun_out/prof_rn${v}_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_rn${v}_bench.log; exit 1; }
  trace=$(find gpurun_out/prof_rn$v -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_steady.py "$trace" momentum_kernel 3 70 > gpurun_out/r3s3_rn_steady_stats$v.txt && head -45 gpurun_out/r3s3_rn_steady_stats$v.txt
  rm -rf gpurun_out/prof_rn$v
done
