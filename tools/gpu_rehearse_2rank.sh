#!/bin/bash
# Rehearsal of the multi-rank bench path (RCCL, sharding stage 3 / DP) with 2 ranks sharing the
# box's single GPU: correctness of the distributed code path, not a scaling measurement.
set -o pipefail
mkdir -p gpurun_out
PADDLE_AMD_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --micro-batch 4 --resnet-batch 64 > gpurun_out/rehearse2.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/rehearse2.log | tail -25
exit $rc
