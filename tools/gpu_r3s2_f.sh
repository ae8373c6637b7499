#!/bin/bash
# staged wgrad + conv epilogues: bitwise tests, then bench A/B (GPT staged9, ResNet conv staged)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "staged or wgrad or grouped or conv" > gpurun_out/t_f.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_f.log; exit 1; }
tail -2 gpurun_out/t_f.log
VAR=PADDLE_AMD_GEMM_STAGED9 VALS="0 1" ROUNDS=2 bash tools/gpu_ab_env.sh
for r in 1 2; do for v in 0 1; do
  PADDLE_AMD_CONV_STAGED=$v timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn_$v.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/rn_$v.log; exit 1; }
  echo "round $r CONV_STAGED=$v $(tail -1 gpurun_out/rn_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
