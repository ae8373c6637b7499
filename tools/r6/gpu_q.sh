#!/bin/bash
# round 6 (q): dQ-from-dS on an LDS-DMA ring: numerics tests + kernel A/B (register-staged vs ring depth 3 / 4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_flash_ds.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 2; do
  DQ_DMA=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$v -o run --output-format csv -- python3 tools/attn_ds_prof.py ds > $O/p$v.log 2>&1 || { echo "prof $v failed"; tail -20 $O/p$v.log; exit 1; }
  echo "== DQ_DMA=$v"; grep -h "dq_from_ds\|dkdv\|delta_kernel" $O/p$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
  rm -f $O/p$v/*kernel_trace.csv
done
