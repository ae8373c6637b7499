#!/bin/bash
# round 4 (k): full GPU test suite, smoke, bench (the round-end contract on the current tree)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4k_gputest.log 2>&1
rc=$?
tail -15 gpurun_out/r4k_gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests aborted rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r4k_smoke.log; exit 1; }
tail -2 gpurun_out/r4k_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4k_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r4k_bench.log; exit 1; }
tail -1 gpurun_out/r4k_bench.log | cut -c1-400
exit $rc
