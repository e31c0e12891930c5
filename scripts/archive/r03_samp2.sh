#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "sample or ensemble or cfg5 or ml" > gpurun_out/r03s_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03s_tests.log; grep -E "^FAILED" gpurun_out/r03s_tests.log | head -5; [ $rc -ne 0 ] && exit $rc
for so in build_variants/t1024.so iib_project_ldpc_codes_amd/libldpc_mi355x.so; do
  LDPC_LIB_PATH=$so timeout -k 10 200 python scripts/diag/sampler_launch.py 64800 1024 2 2>&1 | grep -v amdgpu.ids
  LDPC_LIB_PATH=$so timeout -k 10 200 python scripts/diag/ens_time.py 0.42 4096 2>&1 | grep -v amdgpu.ids
done
LDPC_LIB_PATH=iib_project_ldpc_codes_amd/libldpc_mi355x.so timeout -k 10 200 python scripts/diag/ens_time.py 0.42 16384 2>&1 | grep -v amdgpu.ids
