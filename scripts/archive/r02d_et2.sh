#!/bin/bash
# GPU box: early-stop timing of the headline code with the 1024-thread local-edge layout.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LDPC_LOC_T=1024 ET=1 timeout -k 10 300 python scripts/kbench36.py build_variants/et.so > gpurun_out/et_t1024.log 2>&1 || exit $?
LDPC_LOC_T=1024 timeout -k 10 300 python scripts/kbench36.py build_variants/et.so >> gpurun_out/et_t1024.log 2>&1 || exit $?
cat gpurun_out/et_t1024.log
