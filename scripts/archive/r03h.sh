#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03h_tests.log; grep -E "^FAILED|Error" gpurun_out/r03h_tests.log | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/diag/et_lsb_debug.py 2>&1 | grep -v amdgpu.ids
for spec in "--algo spa --et 1 --post 0" "--algo spa --et 1 --post 1" "--algo minsum --et 1 --post 1" "--algo minsum --et 1 --post 0"; do
  timeout -k 10 120 python scripts/diag/decode_launch.py $spec --warmup 2 --reps 3 2>&1 | grep -v amdgpu.ids | cut -c1-220
done
for s in 0.70 0.78; do
  timeout -k 10 120 python scripts/diag/decode_launch.py --algo spa --et 1 --post 1 --sigma $s --warmup 2 --reps 3 2>&1 | grep -v amdgpu.ids | cut -c1-220
  timeout -k 10 120 python scripts/diag/decode_launch.py --algo spa --et 1 --post 0 --sigma $s --warmup 2 --reps 3 2>&1 | grep -v amdgpu.ids | cut -c1-220
done
