#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/tune_gemms.sh || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_tuned.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log
echo done
