#!/bin/bash
# PMC counters (MFMA busy, waits, clock) of the hand-written GEMM schedules vs hipBLASLt, fc1 shapes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for v in 8 9; do
  GEMM_VARIANT=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/v$v -o run --output-format csv -- python3 tools/gemm_pmc.py > gpurun_out/pmc/v$v.log 2>&1 || { echo "pmc v$v failed"; tail -20 gpurun_out/pmc/v$v.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
