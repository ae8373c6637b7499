#!/bin/bash
# round 6 (w): Llama layer stack with / without the transient K-major weight copies (FLAGS_pa_kmajor_fwd)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6w; mkdir -p $O
for k in 1 0 1 0; do
  FLAGS_pa_kmajor_fwd=$k timeout -k 10 300 python tools/llama_step.py 8 3 > $O/llama_k$k.log 2>&1 || { echo "llama $k failed"; tail -20 $O/llama_k$k.log; exit 1; }
  echo "kmajor_fwd=$k $(grep -v amdgpu $O/llama_k$k.log | tail -1)"
done
