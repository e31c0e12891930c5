#!/bin/bash
# Round 3: all -m gpu tests, then the bench extras (early stop with / without posteriors).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/r03g_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03g_tests.log; grep -E "^FAILED" gpurun_out/r03g_tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/diag/et_lsb_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03g_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r03g_bench.log') if l.startswith('{')][0])
print(d['value'], d['kernel_ms_per_launch']); print(json.dumps(d['extras'])[:1500])"
exit $rc
