#!/bin/bash
# A/B: forward GEMMs on a transient K-major weight copy (default) vs the N-major weight read directly
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for kf in 1 0 1 0; do
  PADDLE_AMD_KMAJOR_FWD=$kf timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/r3s3_kmaj_$kf.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3s3_kmaj_$kf.log; exit 1; }
  echo "kmajor_fwd=$kf $(tail -1 gpurun_out/r3s3_kmaj_$kf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
