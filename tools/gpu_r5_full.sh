#!/bin/bash
# full GPU test suite (one process), then smoke
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/full/tests.log 2>&1
rc=$?
tail -15 gpurun_out/full/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/full/smoke.log
