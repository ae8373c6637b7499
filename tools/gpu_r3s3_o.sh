#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "decode_step_graph or skinny or graph" > gpurun_out/r3s3_t_o.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3_t_o.log; exit 1; }
tail -2 gpurun_out/r3s3_t_o.log
timeout -k 10 300 python -u tools/fmt_decode_bench.py > gpurun_out/r3s3_fmt_decode3.log 2>&1 || { echo "fmt bench failed"; tail -30 gpurun_out/r3s3_fmt_decode3.log; exit 1; }
grep -v amdgpu gpurun_out/r3s3_fmt_decode3.log
