#!/bin/bash
# A/B run during development: captured Momentum step, host LR (PA_AB_HOST_LR, a temporary knob since removed) vs device LR; found the capture-pool aliasing fixed in optimizer/algorithms.py _graph_lr
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, extra env, -k expr
  env $2 timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -q -k "$3" --timeout 120 --timeout-method thread > gpurun_out/r3s4c_$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc"; grep -E "max err|passed|failed" gpurun_out/r3s4c_$1.log | tail -6
  case $rc in 0|1) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
}
T=test_train_step_hip_graph_matches_eager
run host1 PA_AB_HOST_LR=1 $T
run dev1 PA_AB_X=0 $T
run host2 PA_AB_HOST_LR=1 $T
run dev2 PA_AB_X=0 $T
run sched PA_AB_X=0 "lr_scheduler or dropout_adamw_gpt"
