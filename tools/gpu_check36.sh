#!/bin/bash
# rocprofv3 kernel statistics of both benches (current state)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof36 gpurun_out/prof36_rn
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof36 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof36.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof36.log; exit 1; }
tail -1 gpurun_out/prof36.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof36_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2 > gpurun_out/prof36_rn.log 2>&1 || { echo "prof rn failed"; tail -30 gpurun_out/prof36_rn.log; exit 1; }
tail -1 gpurun_out/prof36_rn.log
