#!/bin/bash
# stem BN+ReLU fusion: resnet tests, bench, aten attribution of the remaining elementwise kernels
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "resnet or batchnorm" > gpurun_out/r3s3_t_g.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3_t_g.log; exit 1; }
tail -2 gpurun_out/r3s3_t_g.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3s3_rn_g.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/r3s3_rn_g.log; exit 1; }
  echo "round $r $(tail -1 gpurun_out/r3s3_rn_g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python tools/rn_opprof.py > gpurun_out/r3s3_rn_opprof.log 2>&1 || { echo "opprof failed"; tail -20 gpurun_out/r3s3_rn_opprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3s3_rn_opprof.log | head -60
