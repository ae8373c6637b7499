#!/bin/bash
# round 6 (h): full GPU suite (fused_bn_add_act / inplace passes, ZB static, planner, dtype) + balanced-grid fp8 cast bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -u tools/fp8_cast_bench.py > $O/cast_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/cast_bench.log; exit 1; }
grep -v amdgpu $O/cast_bench.log
