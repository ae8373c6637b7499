#!/bin/bash
# round 6 (t): BN streaming passes in round-robin row order: numerics + ResNet50 step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_hip_conv_routing.py tests/test_hip_ir_passes.py -k "batchnorm or bn or resnet or conv or fused_bn" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/knob_ab_resnet.py > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
grep -v amdgpu $O/ab.log
