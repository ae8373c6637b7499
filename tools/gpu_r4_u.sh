#!/bin/bash
# round 4 (u): block-order group G of the dS backward module (dK/dV + dQ-from-dS kernels)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for G in 0 1 2 4 8; do
  mkdir -p gpurun_out/prof_g$G
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g$G -o run --output-format csv -- python3 tools/attn_ds_prof.py ds $G > gpurun_out/r4u_prof_g$G.log 2>&1 || { echo "prof G=$G failed"; tail -20 gpurun_out/r4u_prof_g$G.log; exit 1; }
  f=$(find gpurun_out/prof_g$G -name "*kernel_stats.csv" | head -1)
  echo "== G=$G"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:4]:
    print(f\"{r['Name'][:60]:60s} avg {float(r['AverageNs'])/1e3:8.1f} us\")
"
  find gpurun_out/prof_g$G -name "*kernel_trace.csv" -delete
done 2>&1 | tee gpurun_out/r4u_pair_group.txt
