#!/bin/bash
# GPU box: every -m gpu test, smoke(), the default bench line, then the headline kernel's
# profile (trace + PMC passes) under TAG (default r02c).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))" > gpurun_out/host.txt
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
[ -n "${SKIP_PROF:-}" ] && exit 0
TAG=${TAG:-r02c} KREGEX=${KREGEX:-bp_loc} ./scripts/profile.sh
