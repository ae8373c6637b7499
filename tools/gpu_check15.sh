#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "batchnorm or resnet50" --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1 || { echo "bn tests failed"; tail -50 gpurun_out/pytest_bn.log; exit 1; }
tail -1 gpurun_out/pytest_bn.log
timeout -k 10 600 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/bench15_rn.log 2>&1 || { echo "rn bench failed"; tail -40 gpurun_out/bench15_rn.log; exit 1; }
tail -1 gpurun_out/bench15_rn.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_rn
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 6 > gpurun_out/prof_rn.log 2>&1 || { echo "rn prof failed"; tail -30 gpurun_out/prof_rn.log; exit 1; }
tail -1 gpurun_out/prof_rn.log
echo done
