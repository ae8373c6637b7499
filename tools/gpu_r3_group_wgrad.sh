#!/bin/bash
# grouped weight gradients: GPU tests, then the GPT-3 1.3B bench A/B (2 rounds)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "grouped or wgrad_side or gpt" > gpurun_out/r3_gputest_group.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3_gputest_group.log; exit 1; }
tail -1 gpurun_out/r3_gputest_group.log
for r in 1 2; do
  for gw in 0 1; do
    PADDLE_AMD_GROUP_WGRAD=$gw timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/r3_bench_gw$gw.log 2>&1 || { echo "bench gw=$gw failed"; tail -20 gpurun_out/r3_bench_gw$gw.log; exit 1; }
    echo "round $r group_wgrad=$gw $(tail -1 gpurun_out/r3_bench_gw$gw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
