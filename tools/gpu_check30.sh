#!/bin/bash
# flash-attention bwd with the dual-use LDS image: numerics, counters, GPT bench
set -o pipefail
mkdir -p gpurun_out/pmc_attn30
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "flash or gpt" --timeout 120 --timeout-method thread > gpurun_out/pytest30.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest30.log; exit 1; }
tail -1 gpurun_out/pytest30.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmc_attn30/p1 -o p1 --output-format csv -- python3 tools/attn_pmc.py > gpurun_out/pmc_attn30/p1.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_attn30/p1.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench30.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench30.log; exit 1; }
tail -1 gpurun_out/bench30.log
