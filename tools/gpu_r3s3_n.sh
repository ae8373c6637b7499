#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fmt_decode_bench.py > gpurun_out/r3s3_fmt_decode2.log 2>&1 || { echo "fmt bench failed"; tail -30 gpurun_out/r3s3_fmt_decode2.log; exit 1; }
grep -v amdgpu gpurun_out/r3s3_fmt_decode2.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s3_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s3_gputest.log; exit 1; }
tail -2 gpurun_out/r3s3_gputest.log
