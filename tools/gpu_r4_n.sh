#!/bin/bash
# round 4 (n): woq unsigned-code dequant + flash paired conversions: tests, woq sweep, same-box A/B
# of the flash change (HEAD flash objects in _lib/ab) on the attention bench and the GPT bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_matmul.py tests/test_hip_flash_ds.py tests/test_hip_flash_ex.py tests/test_hip_flash_wide.py -m gpu -x -q -k "woq or weight_only or flash or ds or wide or ex" --timeout 120 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4n_tests.log; exit 1; }
tail -2 gpurun_out/r4n_tests.log
WOQ_SWEEP=1 timeout -k 10 600 python -u tools/woq_bench.py > gpurun_out/r4n_woq_sweep.log 2>&1 || { echo "woq sweep failed"; tail -30 gpurun_out/r4n_woq_sweep.log; exit 1; }
grep best gpurun_out/r4n_woq_sweep.log
HEADLIB=$PWD/paddlepaddle-paddle_amd/_lib/ab/libpaddle_amd_kernels_head.so
for i in 1 2; do
  for arm in new head; do
    if [ $arm = head ]; then export PADDLE_AMD_KERNEL_LIB=$HEADLIB; else unset PADDLE_AMD_KERNEL_LIB; fi
    FA_DS_AB=0 timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r4n_attn_${arm}_$i.log 2>&1 || { echo "attn $arm failed"; tail -20 gpurun_out/r4n_attn_${arm}_$i.log; exit 1; }
    echo "== attn $arm $i"; grep -v amdgpu.ids gpurun_out/r4n_attn_${arm}_$i.log | head -4
  done
done
for arm in new head; do
  if [ $arm = head ]; then export PADDLE_AMD_KERNEL_LIB=$HEADLIB; else unset PADDLE_AMD_KERNEL_LIB; fi
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-resnet > gpurun_out/r4n_bench_${arm}.log 2>&1 || { echo "bench $arm failed"; tail -20 gpurun_out/r4n_bench_${arm}.log; exit 1; }
  echo "== bench $arm"; tail -1 gpurun_out/r4n_bench_${arm}.log | cut -c1-160
done
