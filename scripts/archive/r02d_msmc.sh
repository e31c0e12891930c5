#!/bin/bash
# GPU box: Monte-Carlo parity tests (incl. min-sum on bp_loc_kernel), then the configs[2]-shape
# Monte-Carlo rate with the in-tree library and build_variants/noms.so (min-sum MC on bp_lds_kernel).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_loc.py tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread -k "mc or loc or minsum or rank" > gpurun_out/msmc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/msmc_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench_mc.py cfg3 > gpurun_out/msmc_bench.log 2>&1 || exit $?
LDPC_LIB_PATH=build_variants/noms.so timeout -k 10 300 python scripts/kbench_mc.py cfg3 >> gpurun_out/msmc_bench.log 2>&1 || exit $?
cat gpurun_out/msmc_bench.log
