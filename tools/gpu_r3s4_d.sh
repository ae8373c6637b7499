#!/bin/bash
# delta fused into the dQ kernel (extended flash-attention backward): numerics, timing, kernel profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_flash_ex.py tests/test_hip_kernels.py -x -q -k "flash or attn or attention" --timeout 120 --timeout-method thread > gpurun_out/r3s4d_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s4d_tests.log; exit 1; }
tail -2 gpurun_out/r3s4d_tests.log
timeout -k 10 300 python tools/attn_ex_bench.py > gpurun_out/r3s4d_attn_ex.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3s4d_attn_ex.log; exit 1; }
cat gpurun_out/r3s4d_attn_ex.log | grep -v amdgpu.ids
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3s4d_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/attn_ex_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r3s4d_prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3s4d_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3s4d_prof -name "*kernel_stats.csv" | head -2
