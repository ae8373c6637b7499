#!/bin/bash
# PMC counters of the flash-attention kernels (one pass per counter group)
set -o pipefail
mkdir -p gpurun_out/pmc_attn
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmc_attn/p1 -o p1 --output-format csv -- python3 tools/attn_pmc.py > gpurun_out/pmc_attn/p1.log 2>&1 || { echo "pass1 failed"; tail -20 gpurun_out/pmc_attn/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc_attn/p2 -o p2 --output-format csv -- python3 tools/attn_pmc.py > gpurun_out/pmc_attn/p2.log 2>&1 || { echo "pass2 failed"; tail -20 gpurun_out/pmc_attn/p2.log; exit 1; }
echo done
