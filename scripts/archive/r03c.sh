#!/bin/bash
# Round 3: full -m gpu suite on the in-tree build, then A/B timing of build_variants/*.so
# (SPA / min-sum, fixed 50 iterations / early stop hard-only), then the iteration-cost split.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03c_tests.log; grep -E "FAILED|Error" gpurun_out/r03c_tests.log | head; [ $rc -ne 0 ] && exit $rc
for cfg in "ALGO=0 ET=0" "ALGO=1 ET=0" "ALGO=0 ET=1" "ALGO=1 ET=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python scripts/kbench36.py build_variants/*.so iib_project_ldpc_codes_amd/libldpc_mi355x.so || exit $?
done > gpurun_out/r03c_ab.log 2>&1
rc=$?; cat gpurun_out/r03c_ab.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/diag/et_cost.py > gpurun_out/r03c_et_cost.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03c_et_cost.log; exit $rc
