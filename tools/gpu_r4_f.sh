#!/bin/bash
# round 4 (f): resnet layout activation diff, flash tests (default dS at D=128), wide flash + fp8 tests, benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/resnet_layout_act_diff.py > gpurun_out/r4f_resnet_act_diff.log 2>&1 || { echo "act diff failed"; tail -30 gpurun_out/r4f_resnet_act_diff.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_resnet_act_diff.log
timeout -k 10 900 python -u -m pytest tests/test_hip_flash_ds.py tests/test_hip_flash_wide.py tests/test_hip_flash_ex.py tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_flash_tests.log 2>&1 || { echo "flash tests failed"; tail -60 gpurun_out/r4f_flash_tests.log; exit 1; }
tail -3 gpurun_out/r4f_flash_tests.log
timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r4f_fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/r4f_fp8_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_fp8_bench.log
FA_SHAPES=wide timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r4f_attn_wide.log 2>&1 || { echo "attn bench failed"; tail -30 gpurun_out/r4f_attn_wide.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_attn_wide.log
WOQ_SWEEP=1 timeout -k 10 300 python -u tools/woq_bench.py > gpurun_out/r4f_woq_sweep.log 2>&1 || { echo "woq sweep failed"; tail -30 gpurun_out/r4f_woq_sweep.log; exit 1; }
grep best gpurun_out/r4f_woq_sweep.log
timeout -k 10 600 python -u tools/conv_r4_bench.py > gpurun_out/r4f_conv_bench.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/r4f_conv_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_conv_bench.log
mkdir -p gpurun_out/prof_ds gpurun_out/prof_rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds -o run --output-format csv -- python3 tools/attn_ds_prof.py ds > gpurun_out/r4f_prof_ds.log 2>&1 || { echo "prof ds failed"; tail -20 gpurun_out/r4f_prof_ds.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rc -o run --output-format csv -- python3 tools/attn_ds_prof.py rc > gpurun_out/r4f_prof_rc.log 2>&1 || { echo "prof rc failed"; tail -20 gpurun_out/r4f_prof_rc.log; exit 1; }
for d in prof_ds prof_rc; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f\"{r['Name'][:90]:90s} n={r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us\")
"; done > gpurun_out/r4f_attn_ds_kstats.txt 2>&1
cat gpurun_out/r4f_attn_ds_kstats.txt
find gpurun_out/prof_ds gpurun_out/prof_rc -name "*kernel_trace.csv" -delete
