#!/bin/bash
# round 6 (o): fused AdamW one-vector-per-lane / temporal accesses: numerics tests, A/B bench, GPT + Llama bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_gpu_sharding_offload.py -k "adam or optim or shard" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u tools/adamw_bench.py > $O/adamw_bench.log 2>&1 || { echo "adamw bench failed"; tail -20 $O/adamw_bench.log; exit 1; }
grep -v amdgpu $O/adamw_bench.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-resnet > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/r6o/bench.log').read().strip().splitlines()[-1])
print('gpt', d['value'], d['ms_per_step'], 'llama', d['llama2_13b']['value'], d['llama2_13b']['ms_per_step'], 'ernie fp8', d['ernie_fp8']['ms_per_step'], 'bf16', d['ernie_fp8']['bf16_ms_per_step'])
PY
