#!/bin/bash
# round 5 (yy): PMC pass over the final tree's GEMM (GPT-3 1.3B fc1 shapes: fwd, dgrad, wgrad; auto schedules)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5yy
GEMM_VARIANT=0 GEMM_LIB=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/r5yy -o run --output-format csv -- python3 tools/gemm_pmc.py > gpurun_out/r5yy/run.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/r5yy/run.log; exit 1; }
f=$(find gpurun_out/r5yy -name "*counter_collection.csv" | head -1)
python3 tools/pmc_clock.py "$f" gemm > gpurun_out/r5yy/summary.txt 2>&1; cat gpurun_out/r5yy/summary.txt | head -60
