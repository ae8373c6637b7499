#!/bin/bash
# round 4 (g): stem v2 (row-blocked, BN stats epilogue) + NCHW BN-parts fix tests, dS backward with
# double-buffered dQ kernel, conv bench, attention kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_conv_routing.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/r4g_conv_tests.log; exit 1; }
tail -3 gpurun_out/r4g_conv_tests.log
timeout -k 10 300 python -u -m pytest tests/test_hip_flash_ds.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_flash_ds.log 2>&1 || { echo "ds tests failed"; tail -60 gpurun_out/r4g_flash_ds.log; exit 1; }
tail -3 gpurun_out/r4g_flash_ds.log
timeout -k 10 300 python -u tools/resnet_layout_act_diff.py > gpurun_out/r4g_resnet_act_diff.log 2>&1 || { echo "act diff failed"; tail -30 gpurun_out/r4g_resnet_act_diff.log; exit 1; }
grep -E "hits|downsample|layer4.2" gpurun_out/r4g_resnet_act_diff.log
timeout -k 10 600 python -u tools/conv_r4_bench.py > gpurun_out/r4g_conv_bench.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/r4g_conv_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4g_conv_bench.log
FA_DS_AB=1 timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r4g_attn_ds_ab.log 2>&1 || { echo "attn ab failed"; tail -30 gpurun_out/r4g_attn_ds_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4g_attn_ds_ab.log
mkdir -p gpurun_out/prof_ds
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds -o run --output-format csv -- python3 tools/attn_ds_prof.py ds > gpurun_out/r4g_prof_ds.log 2>&1 || { echo "prof ds failed"; tail -20 gpurun_out/r4g_prof_ds.log; exit 1; }
f=$(find gpurun_out/prof_ds -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f\"{r['Name'][:90]:90s} n={r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us\")
" > gpurun_out/r4g_attn_ds_kstats.txt 2>&1
cat gpurun_out/r4g_attn_ds_kstats.txt
find gpurun_out/prof_ds -name "*kernel_trace.csv" -delete
