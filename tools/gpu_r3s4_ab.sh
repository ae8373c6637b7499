#!/bin/bash
# same-box A/B of the GPT-3 1.3B bench: kernel library at ef11031 (separate delta pass, 64x64
# transpose) vs HEAD (delta fused into dQ, wide transpose), alternating twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for arm in old new; do
    if [ $arm = old ]; then lib=$GRAFT_REPO_ROOT/ab_old_kernels.so; else lib=""; fi
    PADDLE_AMD_KERNEL_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/r3s4ab_${arm}_$i.log 2>&1 || { echo "bench $arm $i failed"; tail -20 gpurun_out/r3s4ab_${arm}_$i.log; exit 1; }
    echo "$arm $i $(tail -1 gpurun_out/r3s4ab_${arm}_$i.log | cut -c1-120)"
  done
done
