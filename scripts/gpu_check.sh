#!/bin/bash
# GPU box: parity tests, then a short bench.  Stops at the first crash / timeout.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -5 gpurun_out/bench.log
  exit $brc
fi
exit $rc
