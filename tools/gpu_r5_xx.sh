#!/bin/bash
# round 5 (xx): full GPU suite + smoke + default bench (regression check after the FFN epilogue pass, embedding, gradient-slot changes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5xx
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r5xx/tests.log 2>&1
rc=$?
tail -4 gpurun_out/r5xx/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5xx/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5xx/smoke.log; exit 1; }
tail -1 gpurun_out/r5xx/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5xx/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r5xx/bench.log; exit 1; }
grep '^{' gpurun_out/r5xx/bench.log | cut -c1-400
