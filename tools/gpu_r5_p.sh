#!/bin/bash
# round 5 (p): int8 fused_multi_transformer — static quant kernel + FMT int8 numerics, per-Linear latency
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_fmt_int8.py tests/test_hip_quant.py tests/test_static_quantization.py > gpurun_out/r5p/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5p/tests.log; exit 1; }
tail -8 gpurun_out/r5p/tests.log


bash tools/gpu_r5_q.sh
