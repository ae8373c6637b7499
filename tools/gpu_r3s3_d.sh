#!/bin/bash
# im2col row kernel + DPP stats: targeted tests, then ResNet steady profile (stats on) and A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "bn_stats or epi5 or from_parts or batchnorm or resnet or im2col" > gpurun_out/r3s3_t_bn2.log 2>&1 || { echo "bn tests failed"; tail -40 gpurun_out/r3s3_t_bn2.log; exit 1; }
tail -2 gpurun_out/r3s3_t_bn2.log
mkdir -p gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2 > gpurun_out/prof_rn_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -30 gpurun_out/prof_rn_bench.log; exit 1; }
trace=$(find gpurun_out/prof_rn -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" momentum_kernel 3 70 > gpurun_out/r3s3_rn_steady_v2.txt && head -40 gpurun_out/r3s3_rn_steady_v2.txt
rm -rf gpurun_out/prof_rn
for r in 1 2; do for v in 0 1; do
  PADDLE_AMD_CONV_BN_STATS=$v timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3s3_rn_$v.log 2>&1 || { echo "rn bench failed"; tail -20 gpurun_out/r3s3_rn_$v.log; exit 1; }
  echo "round $r BN_STATS=$v $(tail -1 gpurun_out/r3s3_rn_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
