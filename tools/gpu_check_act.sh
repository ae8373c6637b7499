#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/act_bench.py > gpurun_out/act_bench.log 2>&1 || { echo "act bench failed rc=$?"; tail -20 gpurun_out/act_bench.log; exit 1; }
cat gpurun_out/act_bench.log | grep -v amdgpu.ids
timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_gpt_act.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_gpt_act.log; exit 1; }
tail -1 gpurun_out/bench_gpt_act.log
