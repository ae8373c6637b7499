#!/bin/bash
# PMC passes over the flash-attention fwd / dK-dV / dQ kernels (B16 S1024 H16 D128 causal)
set -o pipefail
bash tools/gpu_check29.sh && python3 tools/pmc_summary.py gpurun_out/pmc_attn > gpurun_out/pmc_attn/summary.txt 2>&1
rc=$?
cat gpurun_out/pmc_attn/summary.txt | head -60
exit $rc
