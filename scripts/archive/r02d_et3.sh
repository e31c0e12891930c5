#!/bin/bash
# GPU box: early-stop timing of the headline code at several noise levels across build_variants/.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for s in 0.70 0.78 0.85 0.90; do
  echo "sigma $s" >> gpurun_out/et_sigma.log
  SIGMA=$s ET=1 timeout -k 10 300 python scripts/kbench36.py build_variants/*.so >> gpurun_out/et_sigma.log 2>&1 || exit $?
done
cat gpurun_out/et_sigma.log
