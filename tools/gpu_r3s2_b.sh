#!/bin/bash
# LDS-staged GEMM epilogue: bitwise test vs the register epilogue, then the epilogue-cost table
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "staged or gemm_layouts or gelu_epilogues or epi3" > gpurun_out/t_b.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_b.log; exit 1; }
tail -2 gpurun_out/t_b.log
timeout -k 10 300 python tools/gemm_epi_cost.py > gpurun_out/epi_cost3.log 2>&1 || { echo "epi cost failed"; tail -20 gpurun_out/epi_cost3.log; exit 1; }
grep epi gpurun_out/epi_cost3.log
