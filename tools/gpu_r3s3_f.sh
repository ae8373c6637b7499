#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/im2col_bench.py 256 > gpurun_out/r3s3_im2col_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3s3_im2col_bench.log; exit 1; }
timeout -k 10 200 python tools/im2col_bench.py 32 >> gpurun_out/r3s3_im2col_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3s3_im2col_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3s3_im2col_bench.log
