#!/bin/bash
# round 4 (j): PMC passes over the weight-only int8 decode GEMM vs the bf16 skinny GEMM (ffn1, M = 1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_woq
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_woq/p1 -o p1 --output-format csv -- python3 tools/woq_pmc.py > gpurun_out/pmc_woq/p1.log 2>&1 || { echo "pass1 failed"; tail -20 gpurun_out/pmc_woq/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_woq/p2 -o p2 --output-format csv -- python3 tools/woq_pmc.py > gpurun_out/pmc_woq/p2.log 2>&1 || { echo "pass2 failed"; tail -20 gpurun_out/pmc_woq/p2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_woq > gpurun_out/r4j_woq_pmc.txt 2>&1
cat gpurun_out/r4j_woq_pmc.txt | head -60
find gpurun_out/pmc_woq -name "*.csv" -size +2M -delete
