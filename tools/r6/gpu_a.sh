#!/bin/bash
# round 6 (a): bench on the round-6 tree (distinct batch per step) + GEMM LDS counters + attention PMC
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 420 python3 bench.py --steps 10 --warmup 3 > $O/bench.log 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.log
# GEMM pass: LDS / VALU counters (SQ <= 8, GRBM <= 2)
GEMM_VARIANT=0 GEMM_LIB=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/gemm -o run --output-format csv -- python3 tools/gemm_pmc.py > $O/gemm.log 2>&1 || { echo "gemm pmc failed"; tail -20 $O/gemm.log; exit 1; }
f=$(find $O/gemm -name "*counter_collection.csv" | head -1)
python3 tools/pmc_clock.py "$f" gemm > $O/gemm_summary.txt 2>&1; cat $O/gemm_summary.txt
# attention pass: same counters
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/attn -o run --output-format csv -- python3 tools/attn_pmc.py > $O/attn.log 2>&1 || { echo "attn pmc failed"; tail -20 $O/attn.log; exit 1; }
f=$(find $O/attn -name "*counter_collection.csv" | head -1)
python3 tools/pmc_clock.py "$f" fa > $O/attn_summary.txt 2>&1; cat $O/attn_summary.txt
