#!/bin/bash
# GPU box: sampler parity tests + sampler timing (+ optional ensemble MC timing).
#   ./scripts/samp_check.sh [tag]
T=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "sampler or ensemble" > gpurun_out/t_samp_$T.txt 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_samp_$T.txt; tail -3 gpurun_out/t_samp_$T.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/diag/sampler_time.py ${SIZES:+--sizes $SIZES} iib_project_ldpc_codes_amd/libldpc_mi355x.so > gpurun_out/samp_$T.txt 2>&1
rc=$?; cat gpurun_out/samp_$T.txt; exit $rc
