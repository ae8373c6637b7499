#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "round_split or gemm or gpt" > gpurun_out/r3s3_t_s.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3_t_s.log; exit 1; }
tail -2 gpurun_out/r3s3_t_s.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-resnet > gpurun_out/r3s3_gpt_s.log 2>&1 || { echo "gpt bench failed"; tail -20 gpurun_out/r3s3_gpt_s.log; exit 1; }
  echo "round $r $(tail -1 gpurun_out/r3s3_gpt_s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
mkdir -p gpurun_out/prof_s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-resnet > gpurun_out/prof_s.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_s.log; exit 1; }
trace=$(find gpurun_out/prof_s -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steady.py "$trace" adamw_kernel 3 40 > gpurun_out/r3s3_gpt_steady2.txt && head -8 gpurun_out/r3s3_gpt_steady2.txt && grep -i "gemm9\|splitk" gpurun_out/r3s3_gpt_steady2.txt
rm -rf gpurun_out/prof_s
