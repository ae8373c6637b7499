#!/bin/bash
# wgrad/dgrad side-stream overlap: GPU tests with it on, then the GPT-3 1.3B bench A/B (2 rounds)
set -o pipefail
mkdir -p gpurun_out
PADDLE_AMD_WGRAD_OVERLAP=1 timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "wgrad_side or gpt" --timeout 120 --timeout-method thread > gpurun_out/r3_gputest_overlap.log 2>&1 || { echo "gpu tests (overlap) failed"; tail -40 gpurun_out/r3_gputest_overlap.log; exit 1; }
tail -1 gpurun_out/r3_gputest_overlap.log
for r in 1 2; do
  for ov in 0 1; do
    PADDLE_AMD_WGRAD_OVERLAP=$ov timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/r3_bench_ov$ov.log 2>&1 || { echo "bench ov=$ov failed"; tail -20 gpurun_out/r3_bench_ov$ov.log; exit 1; }
    echo "round $r overlap=$ov $(tail -1 gpurun_out/r3_bench_ov$ov.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
