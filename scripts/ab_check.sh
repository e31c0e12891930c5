#!/bin/bash
# GPU box: parity tests, then interleaved timing of the library builds given in
# $AB (default: every build_variants/*.so) with scripts/kbench.py.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
LIBS=${AB:-$(ls build_variants/*.so)}
for mode in "ALGO=0 ET=0" "ALGO=1 ET=0" "ALGO=0 ET=1"; do
  env $mode timeout -k 10 300 python scripts/kbench.py $LIBS > gpurun_out/kbench.log 2>&1; rc=$?
  echo "kbench $mode rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log | tail -6
  [ $rc -ne 0 ] && exit $rc
done
exit 0
