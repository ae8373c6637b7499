#!/bin/bash
# round 6 (ab): final-tree GPU suite + smoke + bench (after the fp8 bias-from-cast and SOT Layer changes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ab; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/r6ab/bench.log').read().strip().splitlines()[-1])
print('gpt', d['value'], d['ms_per_step'], 'resnet', d['resnet50']['value'], 'llama', d['llama2_13b']['value'], d['llama2_13b']['ms_per_step'], 'ernie fp8', d['ernie_fp8']['ms_per_step'], 'bf16', d['ernie_fp8']['bf16_ms_per_step'], d['ernie_fp8']['fp8_speedup_vs_bf16'])
PY
