#!/bin/bash
# round 5 (e): full bench (GPT-3 1.3B + ResNet50 + llama / ERNIE keys)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e
timeout -k 10 600 python bench.py > gpurun_out/r5e/bench.json 2> gpurun_out/r5e/bench.err || { echo "bench failed"; tail -30 gpurun_out/r5e/bench.err; exit 1; }
cat gpurun_out/r5e/bench.json
