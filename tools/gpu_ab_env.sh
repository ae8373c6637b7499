#!/bin/bash
# A/B of an env switch on the GPT-3 1.3B bench in one process chain on one box:
#   VAR=<name> VALS="0 1" ROUNDS=2 bash tools/gpu_ab_env.sh
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VALS:-0 1}; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:---no-resnet} > gpurun_out/ab_$v.log 2>&1 || { echo "bench $VAR=$v failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
    echo "round $r $VAR=$v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("resnet50", {}).get("value", ""))')"
  done
done
