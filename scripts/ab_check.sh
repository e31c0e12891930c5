set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench.py build_variants/old.so build_variants/new.so > gpurun_out/kbench.log 2>&1; rc=$?
echo "kbench rc=$rc"; cat gpurun_out/kbench.log | tail -5
[ $rc -ne 0 ] && exit $rc
ALGO=1 timeout -k 10 300 python scripts/kbench.py build_variants/old.so build_variants/new.so > gpurun_out/kbench_ms.log 2>&1; rc=$?
echo "kbench ms rc=$rc"; tail -3 gpurun_out/kbench_ms.log
ET=1 timeout -k 10 300 python scripts/kbench.py build_variants/old.so build_variants/new.so > gpurun_out/kbench_et.log 2>&1; rc=$?
echo "kbench et rc=$rc"; tail -3 gpurun_out/kbench_et.log
exit $rc
