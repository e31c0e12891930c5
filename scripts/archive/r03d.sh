#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python scripts/diag/et_lsb_debug.py 2>&1 | grep -v amdgpu.ids
LDPC_LIB_PATH=build_variants/old.so timeout -k 10 120 python scripts/diag/et_lsb_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 300 --timeout-method thread > gpurun_out/r03d_tests.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r03d_tests.log; grep -E "^FAILED" gpurun_out/r03d_tests.log | head -20
