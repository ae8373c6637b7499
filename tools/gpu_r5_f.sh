#!/bin/bash
# round 5 (f): ProgramDesc ERNIE predictor with IR fusion passes: tests, latency, rocprof kernel census
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_hip_ir_passes.py tests/test_hip_quant.py > gpurun_out/r5f/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r5f/tests.log; exit 1; }
tail -2 gpurun_out/r5f/tests.log
timeout -k 10 300 python tools/ernie_predictor.py --no-ir > gpurun_out/r5f/pred_noir.log 2>&1 || { echo "pred noir failed"; tail -30 gpurun_out/r5f/pred_noir.log; exit 1; }
grep ir= gpurun_out/r5f/pred_noir.log
timeout -k 10 300 python tools/ernie_predictor.py > gpurun_out/r5f/pred_ir.log 2>&1 || { echo "pred ir failed"; tail -30 gpurun_out/r5f/pred_ir.log; exit 1; }
grep -E "ir=|max" gpurun_out/r5f/pred_ir.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/prof_ir -o run --output-format csv -- python3 tools/ernie_predictor.py --runs 5 --no-ref > gpurun_out/r5f/prof_ir.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5f/prof_ir.log; exit 1; }
st=$(find gpurun_out/r5f/prof_ir -name "*kernel_stats.csv" | head -1)
python3 - "$st" <<'PY' > gpurun_out/r5f/kernel_census.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("every kernel of a fused-predictor process (export on the CPU, 3 warm-up + 5 timed runs)")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:40]:
    print(f"{int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:9.3f} ms  {r['Name'][:110]}")
PY
head -45 gpurun_out/r5f/kernel_census.txt
rm -f $(find gpurun_out/r5f/prof_ir -name "*kernel_trace.csv")
