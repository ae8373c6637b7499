#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "1024 4 1024" "8192 4 4096" "1024 4 1024" "8192 4 4096" "8192 4 1024"; do
  timeout -k 10 150 python -u tools/ab_act.py $cfg --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/ab.log; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/ab.log | cut -c1-140)"
done
