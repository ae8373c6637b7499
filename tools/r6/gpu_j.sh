#!/bin/bash
# round 6 (j): wave-per-row LayerNorm backward — numerics tests, A/B micro-bench, ERNIE bf16 / fp8 steps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -m gpu -k "layernorm or rmsnorm or dropout_add_norm or norm" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/norm_bwd_ab.py > $O/norm_ab.log 2>&1 || { echo "ab failed"; tail -20 $O/norm_ab.log; exit 1; }
grep -v amdgpu $O/norm_ab.log
for m in fp8 bf16; do
timeout -k 10 300 python tools/ernie_step.py $m 10 3 > $O/ernie_$m.log 2>&1 || { echo "ernie $m failed"; tail -20 $O/ernie_$m.log; exit 1; }
grep -v amdgpu $O/ernie_$m.log | tail -1
done
