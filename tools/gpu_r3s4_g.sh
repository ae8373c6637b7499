#!/bin/bash
# smoke + 2-rank (gloo, one shared GPU) rehearsal of the sharded bench path after the optimizer changes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s4g_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r3s4g_smoke.log; exit 1; }
tail -1 gpurun_out/r3s4g_smoke.log
PADDLE_AMD_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --micro-batch 4 --resnet-batch 64 > gpurun_out/r3s4g_rehearse2.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/r3s4g_rehearse2.log; exit 1; }
tail -1 gpurun_out/r3s4g_rehearse2.log | cut -c1-300
