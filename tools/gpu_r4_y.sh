#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4y_gputest.log 2>&1
rc=$?
tail -4 gpurun_out/r4y_gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests aborted rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4y_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r4y_smoke.log; exit 1; }
tail -1 gpurun_out/r4y_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4y_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r4y_bench.log; exit 1; }
tail -1 gpurun_out/r4y_bench.log | cut -c1-300
exit $rc
exit $rc
