#!/bin/bash
# Round 3: the early-stop / bp_loc GPU tests, then A/B of the early-stop decode (ET=1) and
# Monte-Carlo extras across build_variants/*.so and the in-tree build.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03f_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "ALGO=0 ET=1" "ALGO=1 ET=1" "ALGO=0 ET=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python scripts/kbench36.py build_variants/*.so iib_project_ldpc_codes_amd/libldpc_mi355x.so || exit $?
done 2>&1 | grep -v amdgpu.ids
