#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5i/prof -o run --output-format csv -- python3 tools/attn_mask_prof.py > gpurun_out/r5i/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5i/prof.log; exit 1; }
st=$(find gpurun_out/r5i/prof -name "*kernel_stats.csv" | head -1)
python3 - "$st" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:120]}")
PY
rm -f $(find gpurun_out/r5i/prof -name "*kernel_trace.csv")
