#!/bin/bash
# graph-safe dropout / AdamW powers: graph tests, full GPU suite, GPT bench eager vs --graph
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "graph or dropout or adamw" > gpurun_out/r3s3_t_h.log 2>&1 || { echo "graph tests failed"; tail -40 gpurun_out/r3s3_t_h.log; exit 1; }
tail -2 gpurun_out/r3s3_t_h.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s3_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s3_gputest.log; exit 1; }
tail -2 gpurun_out/r3s3_gputest.log
for r in 1 2; do for gflag in "" "--graph"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-resnet $gflag > gpurun_out/r3s3_gpt_g.log 2>&1 || { echo "gpt bench failed"; tail -20 gpurun_out/r3s3_gpt_g.log; exit 1; }
  echo "round $r graph=[$gflag] $(tail -1 gpurun_out/r3s3_gpt_g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done; done
