#!/bin/bash
# round 6 (z): conv filter gradient with <= 16 pixel splits finished in one pass: numerics + ResNet50 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_hip_conv_routing.py tests/test_conv3d_depth_taps.py -k "conv or wgrad or resnet" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
KNOB=pa_conv_set_wgrad_direct VALUES=1,0 timeout -k 10 400 python -u tools/knob_ab_resnet.py > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
grep -v amdgpu $O/ab.log
