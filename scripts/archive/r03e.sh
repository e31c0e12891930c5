#!/bin/bash
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
for so in build_variants/*.so; do
  LDPC_LIB_PATH=$so timeout -k 10 120 python scripts/diag/et_lsb_debug.py 2>&1 | grep -v amdgpu.ids | head -2
done
