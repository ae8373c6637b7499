#!/bin/bash
# round 6 (f): persistent fp8 cast kernel — bitwise tests, cast micro-bench, ERNIE fp8 vs bf16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_fp8.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -v "^frame\|^  File" $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/fp8_cast_bench.py > $O/cast_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/cast_bench.log; exit 1; }
cat $O/cast_bench.log
for m in fp8 bf16; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > $O/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 $O/ernie_$m.log; exit 1; }
grep -v amdgpu $O/ernie_$m.log | tail -1
done
