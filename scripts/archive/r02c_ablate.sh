#!/bin/bash
# GPU box: headline decode time across the build_variants/ libraries (phase / layout ablations).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/kbench36.py build_variants/*.so > gpurun_out/ablate.log 2>&1
rc=$?; cat gpurun_out/ablate.log; exit $rc
