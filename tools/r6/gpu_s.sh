#!/bin/bash
# round 6 (s): same-box A/B in the GPT bench: dQ-from-dS ring kernel (dq2, default) vs register-staged (dq0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
for mode in dq2 dq0 dq2 dq0; do
  timeout -k 10 300 python -c "
import sys, runpy
import paddle
from paddle.ops import _native
_native._load()
if '$mode' == 'dq0':
    _native.lib.pa_flash_ds_set_dq_dma(0)
sys.argv = ['bench.py', '--no-resnet', '--no-extra', '--steps', '10', '--warmup', '3']
runpy.run_path('bench.py', run_name='__main__')
" > $O/$mode.log 2>&1 || { echo "$mode failed"; tail -20 $O/$mode.log; exit 1; }
  echo "$mode $(tail -1 $O/$mode.log | cut -c1-160)"
done
