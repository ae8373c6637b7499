#!/bin/bash
# GPT-3 1.3B bench step replayed as one captured hipGraph (device learning rate, per-replay hooks)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --graph --steps 20 --warmup 5 --no-resnet > gpurun_out/r3s4i_graph_bench.log 2>&1 || { echo "graph bench failed"; tail -30 gpurun_out/r3s4i_graph_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3s4i_graph_bench.log | tail -3 | cut -c1-400
