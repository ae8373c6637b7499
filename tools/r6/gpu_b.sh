#!/bin/bash
# round 6 (b): ERNIE static step eager vs hipGraph replay (bf16 / fp8)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 400 python3 tools/r6/ernie_graph_ab.py > $O/ernie_graph_ab.log 2>&1; rc=$?
cat $O/ernie_graph_ab.log | grep -v Warning | tail -30
exit $rc
