#!/bin/bash
# PMC pass over the schedule-11 GEMM (fc1 shapes: fwd, dgrad, wgrad) with the clock counter
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc11
GEMM_VARIANT=11 GEMM_LIB=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/pmc11 -o run --output-format csv -- python3 tools/gemm_pmc.py > gpurun_out/pmc11/run.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc11/run.log; exit 1; }
find gpurun_out/pmc11 -name "*.csv" | head
