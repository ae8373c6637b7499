#!/bin/bash
# FMT decode-step kernel profile + full GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_fmt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fmt -o run --output-format csv -- python3 tools/fmt_decode_bench.py > gpurun_out/r3s3_fmt_prof.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/r3s3_fmt_prof.log; exit 1; }
stats=$(find gpurun_out/prof_fmt -name "*kernel_stats.csv" | head -1)
python3 - "$stats" > gpurun_out/r3s3_fmt_kernel_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms over the whole bench (3 batch sizes x 2 arms x 23 steps x 2 layers)")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:110]}")
PY
cat gpurun_out/r3s3_fmt_kernel_stats.txt
rm -rf gpurun_out/prof_fmt
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3s3_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r3s3_gputest.log; exit 1; }
tail -2 gpurun_out/r3s3_gputest.log
