#!/bin/bash
# GPU box: early-stop parity tests on the local-edge kernel, then fixed-count and early-stop
# timing of the headline code across build_variants/.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "early_stop or loc or headline" > gpurun_out/et_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/et_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench36.py build_variants/*.so > gpurun_out/et_fixed.log 2>&1 || exit $?
cat gpurun_out/et_fixed.log
ET=1 timeout -k 10 300 python scripts/kbench36.py build_variants/*.so > gpurun_out/et_et.log 2>&1 || exit $?
cat gpurun_out/et_et.log
