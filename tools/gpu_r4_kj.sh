#!/bin/bash
# round 4 (k + j): full GPU suite, smoke, bench, then the woq PMC passes
set -o pipefail
bash tools/gpu_r4_k.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r4_j.sh
exit $rc
