#!/bin/bash
# round 6 (d): GPU suite + smoke + bench after the paddle DataType change and static TP
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
rc=$?
tail -4 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -3 $O/bench.log
