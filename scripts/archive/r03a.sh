#!/bin/bash
# Round 3, first GPU call: the new parity tests (advisor graph on bp_loc_kernel, multi-rank),
# the 2-rank bench rehearsal on one GPU (gloo), and a short N=1 bench line.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_loc.py tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread -k "check6 or multirank or mc_run" > gpurun_out/r03a_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03a_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 2 --rehearse-on-one-gpu --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03a_bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -c 1500 gpurun_out/r03a_bench2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03a_bench1.log 2>&1
rc=$?; echo "bench1 rc=$rc"; tail -c 3000 gpurun_out/r03a_bench1.log
exit $rc
