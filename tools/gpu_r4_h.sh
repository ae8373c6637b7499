#!/bin/bash
# round 4 (h): woq decode GEMM timed by graph replay (device time), GPT bench, flash-attention PMC
# passes (fwd / dK-dV / dQ-from-dS, B16 S1024 H16 D128 causal)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_attn
timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4h_woq_bench.log 2>&1 || { echo "woq bench failed"; tail -30 gpurun_out/r4h_woq_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4h_woq_bench.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4h_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r4h_bench.log; exit 1; }
tail -2 gpurun_out/r4h_bench.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn/p1 -o p1 --output-format csv -- python3 tools/attn_pmc.py > gpurun_out/pmc_attn/p1.log 2>&1 || { echo "pass1 failed"; tail -20 gpurun_out/pmc_attn/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn/p2 -o p2 --output-format csv -- python3 tools/attn_pmc.py > gpurun_out/pmc_attn/p2.log 2>&1 || { echo "pass2 failed"; tail -20 gpurun_out/pmc_attn/p2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_attn > gpurun_out/r4h_attn_pmc.txt 2>&1
cat gpurun_out/r4h_attn_pmc.txt | head -80
find gpurun_out/pmc_attn -name "*.csv" -size +2M -delete
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn/p3 -o p3 --output-format csv -- python3 tools/attn_pmc.py > gpurun_out/pmc_attn/p3.log 2>&1 || { echo "pass3 failed"; tail -20 gpurun_out/pmc_attn/p3.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_attn > gpurun_out/r4h_attn_pmc.txt 2>&1
cat gpurun_out/r4h_attn_pmc.txt | head -120
find gpurun_out/pmc_attn -name "*.csv" -size +2M -delete
