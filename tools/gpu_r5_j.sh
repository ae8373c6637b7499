#!/bin/bash
# round 5 (j): mask-free dispatch of all-keep batch entries — flash numerics tests, kernel census
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_hip_flash_sp.py tests/test_hip_flash_ex.py tests/test_hip_flash_ds.py > gpurun_out/r5j/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5j/tests.log; exit 1; }
tail -2 gpurun_out/r5j/tests.log
bash tools/gpu_r5_i.sh
