#!/bin/bash
# round 6 (m): GPU suite after the SOT with-block and guard changes + ERNIE steps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for m in fp8 bf16; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > $O/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 $O/ernie_$m.log; exit 1; }
grep -v amdgpu $O/ernie_$m.log | tail -1
done
