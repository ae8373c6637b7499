#!/bin/bash
# round 4 (i): dS^T stored as contiguous [64][128] tiles (dQ-from-dS reads 16 KiB runs): dS tests,
# kernel stats, dS A/B bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_flash_ds.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4t_flash_ds.log 2>&1 || { echo "ds tests failed"; tail -60 gpurun_out/r4t_flash_ds.log; exit 1; }
tail -2 gpurun_out/r4t_flash_ds.log
mkdir -p gpurun_out/prof_ds_t
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds_t -o run --output-format csv -- python3 tools/attn_ds_prof.py ds > gpurun_out/r4t_prof_ds.log 2>&1 || { echo "prof ds failed"; tail -20 gpurun_out/r4t_prof_ds.log; exit 1; }
f=$(find gpurun_out/prof_ds_t -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print(f\"{r['Name'][:90]:90s} n={r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us\")
" > gpurun_out/r4t_attn_ds_kstats.txt 2>&1
cat gpurun_out/r4t_attn_ds_kstats.txt
find gpurun_out/prof_ds_t -name "*kernel_trace.csv" -delete
FA_DS_AB=1 timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r4t_attn_ds_ab.log 2>&1 || { echo "attn ab failed"; tail -30 gpurun_out/r4t_attn_ds_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4t_attn_ds_ab.log
