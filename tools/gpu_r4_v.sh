#!/bin/bash
# round 4 (v): ResNeXt50 NCHW zero-MIOpen step test
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_conv_routing.py -m gpu -x -q -k "resnext" --timeout 240 --timeout-method thread > gpurun_out/r4v_resnext.log 2>&1 || { echo "resnext test failed"; tail -40 gpurun_out/r4v_resnext.log; exit 1; }
tail -2 gpurun_out/r4v_resnext.log
